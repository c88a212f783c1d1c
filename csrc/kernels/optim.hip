// Fused optimizer steps over a flat parameter arena (K4 Adam/AdamW, K5 SGD,
// K6 RMSprop in SURVEY.md section 2.7).
//
// One launch updates every parameter of the model: the framework keeps
// parameters in ONE contiguous fp32 master buffer (+ an optional bf16 model
// copy that the layers read) and gradients in ONE contiguous buffer whose
// slices are the all-reduce buckets.  Each lane moves 8 elements per
// iteration with 16-byte loads/stores; memory-bound by construction
// (Adam: 2 B grad + 12 B state read, 12 B state + 2 B model written / param).
//
// Hyper-parameters are read from a small DEVICE array `hp` so the kernel can
// be captured in a hipGraph and replayed with new learning rates / step
// counts (the host refreshes `hp` with an async H2D copy before each replay).
#include "ca_common.h"

namespace {

template <typename G>
__device__ __forceinline__ void load8(const G* g, long i, float (&out)[8]);

template <>
__device__ __forceinline__ void load8<bf16_t>(const bf16_t* g, long i, float (&out)[8]) {
  us8 v = *reinterpret_cast<const us8*>(g + i);
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = bf2f(v[j]);
}

template <>
__device__ __forceinline__ void load8<float>(const float* g, long i, float (&out)[8]) {
  f4 a = *reinterpret_cast<const f4*>(g + i);
  f4 b = *reinterpret_cast<const f4*>(g + i + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) { out[j] = a[j]; out[j + 4] = b[j]; }
}

__device__ __forceinline__ void ld8f(const float* p, long i, float (&o)[8]) {
  f4 a = *reinterpret_cast<const f4*>(p + i);
  f4 b = *reinterpret_cast<const f4*>(p + i + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) { o[j] = a[j]; o[j + 4] = b[j]; }
}

__device__ __forceinline__ void st8f(float* p, long i, const float (&o)[8]) {
  f4 a, b;
#pragma unroll
  for (int j = 0; j < 4; ++j) { a[j] = o[j]; b[j] = o[j + 4]; }
  *reinterpret_cast<f4*>(p + i) = a;
  *reinterpret_cast<f4*>(p + i + 4) = b;
}

__device__ __forceinline__ void st8bf(bf16_t* p, long i, const float (&o)[8]) {
  us8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = f2bf(o[j]);
  *reinterpret_cast<us8*>(p + i) = v;
}

// zero the 8 gradient elements just consumed (fused zero_grad for the next step)
template <typename G>
__device__ __forceinline__ void zero8(G* g, long i) {
  if constexpr (sizeof(G) == 2) {
    *reinterpret_cast<us8*>(g + i) = us8{0, 0, 0, 0, 0, 0, 0, 0};
  } else {
    *reinterpret_cast<f4*>(g + i) = f4{0.f, 0.f, 0.f, 0.f};
    *reinterpret_cast<f4*>(g + i + 4) = f4{0.f, 0.f, 0.f, 0.f};
  }
}

// Hyper-parameters by value (the per-step path: no host -> device copy, no stream sync)
// or from device memory (hp != null: the hipGraph-capturable path, values refreshed by
// the host before each replay).
struct HpVals {
  float v[8];
};
__device__ __forceinline__ float hpv(const float* hp, const HpVals& hv, int k) { return hp ? hp[k] : hv.v[k]; }

template <typename G> __device__ __forceinline__ float gload(const G* g, long i);
template <> __device__ __forceinline__ float gload<bf16_t>(const bf16_t* g, long i) { return bf2f(g[i]); }
template <> __device__ __forceinline__ float gload<float>(const float* g, long i) { return g[i]; }

// ---------------------------------------------------------------- SGD ----
// hp: [lr, momentum, dampening, weight_decay, grad_scale, first_step]
struct SgdOp {
  float lr, mom, damp, wd, gs; bool first; bool nesterov;
  __device__ __forceinline__ void operator()(float& p, float& m, float g) const {
    g = g * gs + wd * p;
    if (mom != 0.f) {
      m = first ? g : mom * m + (1.f - damp) * g;
      g = nesterov ? g + mom * m : m;
    }
    p -= lr * g;
  }
};

template <typename G>
__global__ void __launch_bounds__(256) sgd_kernel(float* __restrict__ p, G* __restrict__ g,
                                                  float* __restrict__ m, bf16_t* __restrict__ p16,
                                                  const float* __restrict__ hp, HpVals hv, long n, int nesterov,
                                                  int zero_g) {
  SgdOp op{hpv(hp, hv, 0), hpv(hp, hv, 1), hpv(hp, hv, 2), hpv(hp, hv, 3), hpv(hp, hv, 4), hpv(hp, hv, 5) != 0.f,
           nesterov != 0};
  const long nv = n / 8;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long v = (long)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
    const long i = v * 8;
    float pv[8], gv[8], mv[8];
    ld8f(p, i, pv);
    load8<G>(g, i, gv);
    if (zero_g) zero8<G>(g, i);
    if (op.mom != 0.f) ld8f(m, i, mv);
#pragma unroll
    for (int j = 0; j < 8; ++j) op(pv[j], mv[j], gv[j]);
    st8f(p, i, pv);
    if (op.mom != 0.f) st8f(m, i, mv);
    if (p16) st8bf(p16, i, pv);
  }
  for (long i = nv * 8 + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float pp = p[i], mm = op.mom != 0.f ? m[i] : 0.f;
    op(pp, mm, gload<G>(g, i));
    if (zero_g) g[i] = (G)0;
    p[i] = pp;
    if (op.mom != 0.f) m[i] = mm;
    if (p16) p16[i] = f2bf(pp);
  }
}

// --------------------------------------------------------------- Adam ----
// hp: [lr, beta1, beta2, eps, weight_decay, grad_scale, bias_corr1, bias_corr2]
// decoupled != 0 -> AdamW (decay applied to the weight), else L2 into the grad.
struct AdamOp {
  float lr, b1, b2, eps, wd, gs, bc1, bc2; bool decoupled;
  __device__ __forceinline__ void operator()(float& p, float& m, float& v, float g) const {
    g *= gs;
    if (!decoupled) g += wd * p;
    m = b1 * m + (1.f - b1) * g;
    v = b2 * v + (1.f - b2) * g * g;
    const float mhat = m / bc1;
    const float denom = sqrtf(v / bc2) + eps;
    float upd = mhat / denom;
    if (decoupled) upd += wd * p;
    p -= lr * upd;
  }
};

template <typename G>
__global__ void __launch_bounds__(256) adam_kernel(float* __restrict__ p, G* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   bf16_t* __restrict__ p16, const float* __restrict__ hp,
                                                   HpVals hv, long n, int decoupled, int zero_g) {
  AdamOp op{hpv(hp, hv, 0), hpv(hp, hv, 1), hpv(hp, hv, 2), hpv(hp, hv, 3),
            hpv(hp, hv, 4), hpv(hp, hv, 5), hpv(hp, hv, 6), hpv(hp, hv, 7), decoupled != 0};
  const long nv = n / 8;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < nv; t += stride) {
    const long i = t * 8;
    float pv[8], gv[8], mv[8], vv[8];
    ld8f(p, i, pv);
    load8<G>(g, i, gv);
    if (zero_g) zero8<G>(g, i);
    ld8f(m, i, mv);
    ld8f(v, i, vv);
#pragma unroll
    for (int j = 0; j < 8; ++j) op(pv[j], mv[j], vv[j], gv[j]);
    st8f(p, i, pv);
    st8f(m, i, mv);
    st8f(v, i, vv);
    if (p16) st8bf(p16, i, pv);
  }
  for (long i = nv * 8 + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float pp = p[i], mm = m[i], vv = v[i];
    op(pp, mm, vv, gload<G>(g, i));
    if (zero_g) g[i] = (G)0;
    p[i] = pp; m[i] = mm; v[i] = vv;
    if (p16) p16[i] = f2bf(pp);
  }
}

// ------------------------------------------------------------ RMSprop ----
// hp: [lr, rho, eps, weight_decay, grad_scale, momentum]   (Keras semantics:
// eps added inside the sqrt-free denominator: p -= lr * g / (sqrt(ms) + eps))
struct RmsOp {
  float lr, rho, eps, wd, gs, mom;
  __device__ __forceinline__ void operator()(float& p, float& ms, float& buf, float g) const {
    g = g * gs + wd * p;
    ms = rho * ms + (1.f - rho) * g * g;
    const float upd = g / (sqrtf(ms) + eps);
    if (mom != 0.f) {
      buf = mom * buf + upd;
      p -= lr * buf;
    } else {
      p -= lr * upd;
    }
  }
};

template <typename G>
__global__ void __launch_bounds__(256) rmsprop_kernel(float* __restrict__ p, G* __restrict__ g,
                                                      float* __restrict__ ms, float* __restrict__ buf,
                                                      bf16_t* __restrict__ p16, const float* __restrict__ hp,
                                                      HpVals hv, long n, int zero_g) {
  RmsOp op{hpv(hp, hv, 0), hpv(hp, hv, 1), hpv(hp, hv, 2), hpv(hp, hv, 3), hpv(hp, hv, 4), hpv(hp, hv, 5)};
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float pp = p[i], s = ms[i], b = buf ? buf[i] : 0.f;
    op(pp, s, b, gload<G>(g, i));
    if (zero_g) g[i] = (G)0;
    p[i] = pp; ms[i] = s;
    if (buf) buf[i] = b;
    if (p16) p16[i] = f2bf(pp);
  }
}

// --------------------------------------------------- grad global norm ----
// out[0] += sum(g^2) (fp32 atomics, one per block after an LDS reduction).
template <typename G>
__global__ void __launch_bounds__(256) sumsq_kernel(const G* __restrict__ g, long n, float* __restrict__ out) {
  float acc = 0.f;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float x = gload<G>(g, i);
    acc += x * x;
  }
  acc = wave_sum(acc);
  __shared__ float red[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, red[0] + red[1] + red[2] + red[3]);
}

// g *= scale[0] (scale read from device memory; used for clip-by-global-norm)
template <typename G>
__global__ void __launch_bounds__(256) scale_kernel(G* __restrict__ g, long n, const float* __restrict__ s);

template <>
__global__ void __launch_bounds__(256) scale_kernel<float>(float* __restrict__ g, long n, const float* __restrict__ s) {
  const float k = s[0];
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) g[i] *= k;
}
template <>
__global__ void __launch_bounds__(256) scale_kernel<bf16_t>(bf16_t* __restrict__ g, long n, const float* __restrict__ s) {
  const float k = s[0];
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) g[i] = f2bf(bf2f(g[i]) * k);
}

}  // namespace

// ------------------------------------------------------------ launchers --
extern "C" {

static HpVals hp_vals(const float* hv, int k) {
  HpVals h{};
  for (int i = 0; i < k && i < 8 && hv; ++i) h.v[i] = hv[i];
  return h;
}

// hp: device hyper-parameters (graph-capturable path) or null, then hv (host array) is
// passed by value; zero_g: also zero the gradient elements consumed (fused zero_grad).
int ca_sgd_step(float* p, void* g, int g_is_bf16, float* m, bf16_t* p16, const float* hp, const float* hv, long n,
                int nesterov, int zero_g, hipStream_t s) {
  const int B = 256, G = ca_stream_grid(n / 8 + 1, B);
  const HpVals h = hp_vals(hv, 6);
  if (g_is_bf16)
    sgd_kernel<bf16_t><<<G, B, 0, s>>>(p, (bf16_t*)g, m, p16, hp, h, n, nesterov, zero_g);
  else
    sgd_kernel<float><<<G, B, 0, s>>>(p, (float*)g, m, p16, hp, h, n, nesterov, zero_g);
  CA_LAUNCH_CHECK();
  return 0;
}

int ca_adam_step(float* p, void* g, int g_is_bf16, float* m, float* v, bf16_t* p16, const float* hp, const float* hv,
                 long n, int decoupled, int zero_g, hipStream_t s) {
  const int B = 256, G = ca_stream_grid(n / 8 + 1, B);
  const HpVals h = hp_vals(hv, 8);
  if (g_is_bf16)
    adam_kernel<bf16_t><<<G, B, 0, s>>>(p, (bf16_t*)g, m, v, p16, hp, h, n, decoupled, zero_g);
  else
    adam_kernel<float><<<G, B, 0, s>>>(p, (float*)g, m, v, p16, hp, h, n, decoupled, zero_g);
  CA_LAUNCH_CHECK();
  return 0;
}

int ca_rmsprop_step(float* p, void* g, int g_is_bf16, float* ms, float* buf, bf16_t* p16, const float* hp,
                    const float* hv, long n, int zero_g, hipStream_t s) {
  const int B = 256, G = ca_stream_grid(n, B);
  const HpVals h = hp_vals(hv, 6);
  if (g_is_bf16)
    rmsprop_kernel<bf16_t><<<G, B, 0, s>>>(p, (bf16_t*)g, ms, buf, p16, hp, h, n, zero_g);
  else
    rmsprop_kernel<float><<<G, B, 0, s>>>(p, (float*)g, ms, buf, p16, hp, h, n, zero_g);
  CA_LAUNCH_CHECK();
  return 0;
}

int ca_sumsq(const void* g, int g_is_bf16, long n, float* out, hipStream_t s) {
  const int B = 256, G = ca_stream_grid(n, B);
  if (g_is_bf16)
    sumsq_kernel<bf16_t><<<G, B, 0, s>>>((const bf16_t*)g, n, out);
  else
    sumsq_kernel<float><<<G, B, 0, s>>>((const float*)g, n, out);
  CA_LAUNCH_CHECK();
  return 0;
}

int ca_scale(void* g, int g_is_bf16, long n, const float* scale, hipStream_t s) {
  const int B = 256, G = ca_stream_grid(n, B);
  if (g_is_bf16)
    scale_kernel<bf16_t><<<G, B, 0, s>>>((bf16_t*)g, n, scale);
  else
    scale_kernel<float><<<G, B, 0, s>>>((float*)g, n, scale);
  CA_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
