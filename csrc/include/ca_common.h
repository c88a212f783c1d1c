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

// BatchNorm transforms with a FIXED evaluation order (explicit FMAs).  Every kernel that applies
// one BatchNorm -- the separate passes (bn.hip, pool.hip) and the GEMM operand fetches that fold
// it (ca_gemm_xa.h) -- must round identically; left to -ffp-contract, `A*d + B*x + D` contracts
// differently from one template instantiation to the next.
__device__ __forceinline__ float bn_affine(float x, float scale, float shift) { return __builtin_fmaf(x, scale, shift); }
__device__ __forceinline__ float bn_bwd_affine(float a, float d, float b, float x, float dd) {
  return __builtin_fmaf(a, d, __builtin_fmaf(b, x, dd));
}

// Wave-wide sum / max, every lane gets the result.  DPP within each 16-lane row (row_ror 8 / 4,
// quad swaps: VALU ops, no LDS permutes), then the four row totals read as scalars in a fixed
// order -- against six ds_bpermute round trips of the __shfl_xor butterfly.
#define CA_DPP(v, ctrl) __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), (ctrl), 0xf, 0xf, false))
__device__ __forceinline__ float wave_sum(float v) {
  v += CA_DPP(v, 0x128);  // row_ror:8
  v += CA_DPP(v, 0x124);  // row_ror:4
  v += CA_DPP(v, 0x4e);   // quad_perm [2,3,0,1]
  v += CA_DPP(v, 0xb1);   // quad_perm [1,0,3,2]
  return (__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)) +
          __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16))) +
         (__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32)) +
          __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48)));
}

__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, CA_DPP(v, 0x128));
  v = fmaxf(v, CA_DPP(v, 0x124));
  v = fmaxf(v, CA_DPP(v, 0x4e));
  v = fmaxf(v, CA_DPP(v, 0xb1));
  return fmaxf(fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)),
                     __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16))),
               fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32)),
                     __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48))));
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
