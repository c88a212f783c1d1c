// Sequence-classification head (BERT pooler output -> dropout -> linear classifier) as two
// small kernels instead of a chain of framework elementwise ops (K13 head, reference
// TFC/examples BERT fine-tuning via tf-models' classifier).
//
//   forward : logits[b][l] = sum_c drop(pooled[b][c]) * Wc[l][c] + bc[l]       (fp32 out)
//   backward: dpre[b][c]  = (sum_l dlogits[b][l] Wc[l][c]) * drop'(b, c) * (1 - pooled^2)
//             dWc[l][c]  += sum_b dlogits[b][l] * drop(pooled[b][c])
//             dbc[l]     += sum_b dlogits[b][l]
// pooled = tanh(pre) is the bf16 output of the pooler GEMM epilogue; the backward's tanh'
// uses it as the fused epilogue did.  The dropout mask is the stateless hash of ca_rng.h
// (element index b * C + c), regenerated in the backward.  Both kernels are deterministic
// (fixed summation orders, one writer per output).  L (labels) <= HEAD_LMAX.
#include "ca_common.h"
#include "ca_rng.h"

namespace {

constexpr int HEAD_LMAX = 16;

// one wave per example row
// LM = compile-time bound on the label count L (runtime)
template <int LM>
__global__ void __launch_bounds__(256) cls_head_fwd_kernel(const bf16_t* __restrict__ pooled, long ldp,
                                                           const float* __restrict__ wc, const float* __restrict__ bc,
                                                           float* __restrict__ logits, int B, int C, int L, DropCfg d) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  float acc[LM];
#pragma unroll
  for (int l = 0; l < LM; ++l) acc[l] = 0.f;
  for (int c = lane; c < C; c += 64) {
    float v = bf2f(pooled[(long)b * ldp + c]);
    if (d.on) v *= drop_mul(d, (uint64_t)b * C + c);
#pragma unroll
    for (int l = 0; l < LM; ++l)
      if (l < L) acc[l] += v * wc[(long)l * C + c];
  }
#pragma unroll
  for (int l = 0; l < LM; ++l) {
    if (l < L) {  // L is uniform: every lane takes the same branch
      const float t = wave_sum(acc[l]);
      if (lane == 0) logits[(long)b * L + l] = t + bc[l];
    }
  }
}

// one thread per hidden column, looping over the examples in order
template <int LM>
__global__ void __launch_bounds__(256) cls_head_bwd_kernel(const float* __restrict__ dlogits,
                                                           const bf16_t* __restrict__ pooled, long ldp,
                                                           const float* __restrict__ wc, bf16_t* __restrict__ dpre,
                                                           float* __restrict__ gwc, float* __restrict__ gbc, int B,
                                                           int C, int L, DropCfg d) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x < L && gbc) {
    float t = 0.f;
    for (int b = 0; b < B; ++b) t += dlogits[(long)b * L + threadIdx.x];
    gbc[threadIdx.x] += t;
  }
  if (c >= C) return;
  float w[LM], gw[LM];
#pragma unroll
  for (int l = 0; l < LM; ++l) {
    w[l] = l < L ? wc[(long)l * C + c] : 0.f;
    gw[l] = 0.f;
  }
#pragma unroll 4
  for (int b = 0; b < B; ++b) {
    const float y = bf2f(pooled[(long)b * ldp + c]);
    const float m = d.on ? drop_mul(d, (uint64_t)b * C + c) : 1.f;
    float dp = 0.f;
#pragma unroll
    for (int l = 0; l < LM; ++l) {
      const float dl = l < L ? dlogits[(long)b * L + l] : 0.f;
      dp += dl * w[l];
      gw[l] += dl * (y * m);
    }
    dpre[(long)b * C + c] = f2bf(dp * m * (1.f - y * y));
  }
  if (gwc) {
#pragma unroll
    for (int l = 0; l < LM; ++l)
      if (l < L) gwc[(long)l * C + c] += gw[l];
  }
}

template <int LM>
void head_fwd_l(const bf16_t* pooled, long ldp, const float* wc, const float* bc, float* logits, int B, int C, int L,
                DropCfg d, hipStream_t s) {
  cls_head_fwd_kernel<LM><<<ca_cdiv(B, 4), 256, 0, s>>>(pooled, ldp, wc, bc, logits, B, C, L, d);
}
template <int LM>
void head_bwd_l(const float* dl, const bf16_t* pooled, long ldp, const float* wc, bf16_t* dpre, float* gwc, float* gbc,
                int B, int C, int L, DropCfg d, hipStream_t s) {
  cls_head_bwd_kernel<LM><<<ca_cdiv(C, 256), 256, 0, s>>>(dl, pooled, ldp, wc, dpre, gwc, gbc, B, C, L, d);
}

}  // namespace

extern "C" {

int ca_cls_head_max_labels() { return HEAD_LMAX; }

int ca_cls_head_fwd(const bf16_t* pooled, long ldp, const float* wc, const float* bc, float* logits, int B, int C,
                    int L, float p, uint64_t seed, hipStream_t s) {
  if (B <= 0 || C <= 0 || L <= 0 || L > HEAD_LMAX) return -1;
  const DropCfg d = make_drop(p, seed);
  if (L <= 4) head_fwd_l<4>(pooled, ldp, wc, bc, logits, B, C, L, d, s);
  else head_fwd_l<16>(pooled, ldp, wc, bc, logits, B, C, L, d, s);
  CA_LAUNCH_CHECK();
  return 0;
}

int ca_cls_head_bwd(const float* dlogits, const bf16_t* pooled, long ldp, const float* wc, bf16_t* dpre, float* gwc,
                    float* gbc, int B, int C, int L, float p, uint64_t seed, hipStream_t s) {
  if (B <= 0 || C <= 0 || L <= 0 || L > HEAD_LMAX) return -1;
  const DropCfg d = make_drop(p, seed);
  if (L <= 4) head_bwd_l<4>(dlogits, pooled, ldp, wc, dpre, gwc, gbc, B, C, L, d, s);
  else head_bwd_l<16>(dlogits, pooled, ldp, wc, dpre, gwc, gbc, B, C, L, d, s);
  CA_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
