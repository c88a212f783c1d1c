// Fused softmax + sparse categorical cross-entropy, forward AND backward in
// one pass (K3 + K12 in SURVEY.md section 2.7).
//
// One wave per row.  For each row: max (and argmax, for accuracy), log-sum-exp,
// loss = lse - z[label], dlogits = (softmax - onehot) * grad_scale, where
// grad_scale = 1/global_batch implements Keras' compute_average_loss /
// SUM_OVER_BATCH_SIZE reduction (reference mnist_example_using_ctl.py:93-101).
// The loss row values and a correct-prediction flag are written for metrics.
#include "ca_common.h"

namespace {

template <typename T> __device__ __forceinline__ float ld(const T* p, long i);
template <> __device__ __forceinline__ float ld<float>(const float* p, long i) { return p[i]; }
template <> __device__ __forceinline__ float ld<bf16_t>(const bf16_t* p, long i) { return bf2f(p[i]); }
template <typename T> __device__ __forceinline__ void st(T* p, long i, float v);
template <> __device__ __forceinline__ void st<float>(float* p, long i, float v) { p[i] = v; }
template <> __device__ __forceinline__ void st<bf16_t>(bf16_t* p, long i, float v) { p[i] = f2bf(v); }

template <typename T>
__global__ void __launch_bounds__(256) xent_kernel(const T* __restrict__ z, const int64_t* __restrict__ labels,
                                                  int B, int C, float grad_scale, float label_smoothing,
                                                  float* __restrict__ loss, float* __restrict__ correct,
                                                  T* __restrict__ dz) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const T* zr = z + (long)row * C;
  float m = -INFINITY;
  int am = 0;
  for (int c = lane; c < C; c += 64) {
    float v = ld<T>(zr, c);
    if (v > m) { m = v; am = c; }
  }
  // wave argmax (ties -> smallest index)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float om = __shfl_xor(m, o, 64);
    int oa = __shfl_xor(am, o, 64);
    if (om > m || (om == m && oa < am)) { m = om; am = oa; }
  }
  float s = 0.f, sz = 0.f;
  for (int c = lane; c < C; c += 64) {
    float v = ld<T>(zr, c);
    s += __expf(v - m);
    sz += v;
  }
  s = wave_sum(s);
  sz = wave_sum(sz);
  const float lse = m + __logf(s);
  const long lab = labels[row];
  const bool valid = lab >= 0 && lab < C;
  const float zl = valid ? ld<T>(zr, lab) : 0.f;
  const float eps = label_smoothing;
  // smoothed target: (1-eps)*onehot + eps/C
  const float row_loss = valid ? (1.f - eps) * (lse - zl) + eps * (lse - sz / (float)C) : 0.f;
  if (lane == 0) {
    if (loss) loss[row] = row_loss;
    if (correct) correct[row] = (valid && am == lab) ? 1.f : 0.f;
  }
  if (dz) {
    T* dr = dz + (long)row * C;
    const float inv_s = 1.f / s;
    for (int c = lane; c < C; c += 64) {
      float p = __expf(ld<T>(zr, c) - m) * inv_s;
      float t = (valid ? ((c == lab) ? (1.f - eps) : 0.f) + eps / (float)C : 0.f);
      st<T>(dr, c, valid ? (p - t) * grad_scale : 0.f);
    }
  }
}

}  // namespace

extern "C" int ca_softmax_xent(const void* logits, int is_bf16, const int64_t* labels, int B, int C,
                               float grad_scale, float label_smoothing, float* loss, float* correct,
                               void* dlogits, hipStream_t s) {
  dim3 grid(ca_cdiv(B, 4));
  if (is_bf16)
    xent_kernel<bf16_t><<<grid, 256, 0, s>>>((const bf16_t*)logits, labels, B, C, grad_scale, label_smoothing,
                                             loss, correct, (bf16_t*)dlogits);
  else
    xent_kernel<float><<<grid, 256, 0, s>>>((const float*)logits, labels, B, C, grad_scale, label_smoothing,
                                            loss, correct, (float*)dlogits);
  CA_LAUNCH_CHECK();
  return 0;
}
