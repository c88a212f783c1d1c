// Common device helpers for cloud_amd gfx950 kernels.
//
// Conventions (all kernels):
//   * bf16 tensors are carried as `uint16_t` storage; math in fp32.
//   * vector memory access is 16 B per lane (8 x bf16 or 4 x fp32) -- Guideline 13.
//   * wave = 64 lanes; block sizes are multiples of 64.
//   * every launcher takes a hipStream_t and never allocates or synchronises,
//     so it can be captured into a hipGraph -- except in the debug mode below.
//   * CLOUD_AMD_DEBUG_SYNC=1: every launch is followed by hipDeviceSynchronize(), so a
//     kernel fault is reported by the launcher (and the Python op) that caused it
//     instead of by a later, unrelated call (not usable with graphs).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

inline bool ca_debug_sync() {
  static const bool on = [] {
    const char* e = getenv("CLOUD_AMD_DEBUG_SYNC");
    return e && e[0] == '1';
  }();
  return on;
}

#define CA_WAVE 64

#define CA_HIP_CHECK(expr)                                                     \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    if (_e != hipSuccess) return (int)_e;                                      \
  } while (0)

#define CA_LAUNCH_CHECK()                                                      \
  do {                                                                         \
    hipError_t _le = hipGetLastError();                                        \
    if (_le == hipSuccess && ca_debug_sync()) _le = hipDeviceSynchronize();    \
    if (_le != hipSuccess) return (int)_le;                                    \
  } while (0)

typedef uint16_t bf16_t;
typedef unsigned short us8 __attribute__((ext_vector_type(8)));
typedef unsigned short us4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(bf16_t u) {
  return __uint_as_float(((uint32_t)u) << 16);
}

// Round-to-nearest-even via the native conversion (v_cvt_pk_bf16_f32 at -O3;
// keeps NaN a NaN -- MI355X_MICROARCH "Correctness boundaries").
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

static inline int ca_cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// Grid size for grid-stride memory-bound kernels: enough blocks to fill
// 256 CUs several times over, capped (Guideline 11).
static inline int ca_stream_grid(long work_items, int block) {
  long g = (work_items + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}
