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

// Whole-batch variant for small batches (Keras fit, BERT fine-tuning, the ResNet head):
// ONE block of 16 waves walks the rows (wave w: rows w, w + 16, ...), then reduces the
// per-wave loss / correct partials in a fixed order and writes the MEAN loss (x grad_scale)
// itself, and optionally adds [sum loss, sum correct, rows] * acc_w into a device metric
// accumulator -- the loss's sum / divide kernels and the metrics' argmax / compare /
// reduce kernels (and their host syncs) are gone from the step.  Deterministic.
template <typename T>
__global__ void __launch_bounds__(1024) xent_batch_kernel(const T* __restrict__ z, long ldz,
                                                         const int64_t* __restrict__ labels,
                                                         int B, int C, float grad_scale, float label_smoothing,
                                                         float* __restrict__ mean_out, float* __restrict__ correct,
                                                         T* __restrict__ dz, float* __restrict__ acc, float acc_w) {
  __shared__ float red[16][2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float wl = 0.f, wc = 0.f;
  for (int row = wave; row < B; row += 16) {
    const T* zr = z + (long)row * ldz;  // logits rows may be strided (a padded head's [:, :C] view)
    float m = -INFINITY;
    int am = 0;
    for (int c = lane; c < C; c += 64) {
      const float v = ld<T>(zr, c);
      if (v > m) { m = v; am = c; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float om = __shfl_xor(m, o, 64);
      const int oa = __shfl_xor(am, o, 64);
      if (om > m || (om == m && oa < am)) { m = om; am = oa; }
    }
    float s = 0.f, sz = 0.f;
    for (int c = lane; c < C; c += 64) {
      const float v = ld<T>(zr, c);
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
    const float row_loss = valid ? (1.f - eps) * (lse - zl) + eps * (lse - sz / (float)C) : 0.f;
    const float ok = (valid && am == lab) ? 1.f : 0.f;
    wl += row_loss;
    wc += ok;
    if (lane == 0 && correct) correct[row] = ok;
    if (dz) {
      T* dr = dz + (long)row * C;
      const float inv_s = 1.f / s;
      for (int c = lane; c < C; c += 64) {
        const float p = __expf(ld<T>(zr, c) - m) * inv_s;
        const float t = (valid ? ((c == lab) ? (1.f - eps) : 0.f) + eps / (float)C : 0.f);
        st<T>(dr, c, valid ? (p - t) * grad_scale : 0.f);
      }
    }
  }
  if (lane == 0) {
    red[wave][0] = wl;
    red[wave][1] = wc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float tl = 0.f, tc = 0.f;
    for (int w = 0; w < 16; ++w) {
      tl += red[w][0];
      tc += red[w][1];
    }
    mean_out[0] = tl * grad_scale;
    if (acc) {
      acc[0] += tl * acc_w;
      acc[1] += tc * acc_w;
      acc[2] += (float)B * acc_w;
    }
  }
}

}  // namespace

extern "C" int ca_softmax_xent_batch(const void* logits, long ldz, int is_bf16, const int64_t* labels, int B, int C,
                                     float grad_scale, float label_smoothing, float* mean_out, float* correct,
                                     void* dlogits, float* acc, float acc_w, hipStream_t s) {
  if (B <= 0 || C <= 0 || ldz < C) return -1;
  if (is_bf16)
    xent_batch_kernel<bf16_t><<<1, 1024, 0, s>>>((const bf16_t*)logits, ldz, labels, B, C, grad_scale,
                                                label_smoothing, mean_out, correct, (bf16_t*)dlogits, acc, acc_w);
  else
    xent_batch_kernel<float><<<1, 1024, 0, s>>>((const float*)logits, ldz, labels, B, C, grad_scale,
                                               label_smoothing, mean_out, correct, (float*)dlogits, acc, acc_w);
  CA_LAUNCH_CHECK();
  return 0;
}

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
