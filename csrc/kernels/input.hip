// Input-layer conversion (K9 in SURVEY.md 2.7): uint8 NHWC images straight from the
// host loader (cloud_amd/data) -> normalised bf16 NHWC on the GPU,
//   y = (x - mean[c]) * inv_std[c],  c = element index mod C (C <= 8),
// so the host moves 1 byte per element over PCIe and never does float math.
// One thread handles 16 consecutive bytes (one 16-B load, two 16-B stores).
#include "ca_common.h"

namespace {

struct ChanParams {
  float mean[8];
  float inv_std[8];
};

__global__ void __launch_bounds__(256) u8_normalize_kernel(const uint8_t* __restrict__ x, bf16_t* __restrict__ y,
                                                           long n, int C, ChanParams cp) {
  const long i0 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 16;
  if (i0 >= n) return;
  if (i0 + 16 <= n) {
    typedef unsigned char u8x16 __attribute__((ext_vector_type(16)));
    const u8x16 v = *reinterpret_cast<const u8x16*>(x + i0);
    us8 lo, hi;
    int c = (int)(i0 % C);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float f = ((float)v[j] - cp.mean[c]) * cp.inv_std[c];
      if (j < 8) lo[j] = f2bf(f);
      else hi[j - 8] = f2bf(f);
      c = (c + 1 == C) ? 0 : c + 1;
    }
    reinterpret_cast<us8*>(y + i0)[0] = lo;
    reinterpret_cast<us8*>(y + i0)[1] = hi;
    return;
  }
  for (long i = i0; i < n; ++i) {
    const int c = (int)(i % C);
    y[i] = f2bf(((float)x[i] - cp.mean[c]) * cp.inv_std[c]);
  }
}

}  // namespace

extern "C" {

// x: n bytes (n % C == 0, x and y 16-B aligned); mean / std: C floats (host memory).
int ca_u8_normalize(const uint8_t* x, bf16_t* y, long n, int C, const float* mean, const float* std_,
                    hipStream_t s) {
  if (C < 1 || C > 8 || n % C != 0) return -1;
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) return -1;
  ChanParams cp;
  for (int c = 0; c < 8; ++c) {
    cp.mean[c] = c < C ? mean[c] : 0.f;
    cp.inv_std[c] = c < C ? 1.f / std_[c] : 1.f;
  }
  const long threads = (n + 15) / 16;
  u8_normalize_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, s>>>(x, y, n, C, cp);
  CA_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
