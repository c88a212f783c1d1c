// Fused multi-head attention (K13 in SURVEY.md 2.7) for head_dim 64 on MFMA.
//
// Layout: the QKV projection output qkv[B*S][3*H*64] (Q | K | V, head h at
// columns h*64 inside each third) is consumed in place -- no head split /
// transpose copies; the context is written to ctx[B*S][H*64].
//
// Forward (one workgroup = 64 queries of one (batch, head), 4 waves x 16 rows):
//   S = Q K^T * scale over 64-key blocks, online softmax in registers (exp2
//   domain), key-padding mask from key_len[b], attention-probability dropout
//   from the stateless hash (ca_rng.h), O += P V; P goes C-layout -> LDS -> A
//   fragments (one 2.3 KB slab per wave).  Log-sum-exp per row is kept for
//   the backward.  Q fragments are loaded straight from HBM into registers.
//
// Backward = three kernels, no atomics:
//   prep : Dv[q] = rowsum(dO * O)
//   dKV  : per 64-key block, loop over query blocks: S^T, P^T, dV += Pd^T dO,
//          dP^T = V dO^T, dS^T = P^T (dP^T*mask - Dv), dK += dS^T Q
//   dQ   : per 64-query block, loop over key blocks: dQ += dS K
// MFMA: v_mfma_f32_16x16x32_bf16; K-contiguous operands via ds_read_b128,
// N-contiguous ones (V / dO / Q / K as B with k along rows) via ds_read_b64_tr_b16.
#include "ca_mfma_core.h"
#include "ca_rng.h"

namespace {
using namespace ca;

constexpr int D = 64;     // head dim
constexpr int QB = 64;    // queries per workgroup
constexpr int KB = 64;    // keys per block
constexpr int LDT = 72;   // LDS row pitch (64 + 8 pad) of every 64x64 tile
constexpr int PLD = 72;   // per-wave P / dS slab pitch
constexpr float LOG2E = 1.4426950408889634f;

__device__ __forceinline__ void tile_load(short* lds, const bf16_t* g, long ld, int tid) {
  // 64 rows x 64 bf16 (8 chunks of 16 B per row): 512 chunks, 2 per thread
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tid + i * 256;
    const int r = c >> 3, col = (c & 7) * 8;
    *reinterpret_cast<s8v*>(lds + r * LDT + col) = *reinterpret_cast<const s8v*>(g + (long)r * ld + col);
  }
}

// C-layout 16x64 fp32 (4 tiles) -> bf16 slab [16][PLD] of this wave
__device__ __forceinline__ void slab_store(short* slab, const f4v (&v)[4], int lane) {
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) slab[((lane >> 4) * 4 + r) * PLD + t * 16 + (lane & 15)] = (short)f2bf(v[t][r]);
}

// A fragment (16 rows x 32 k, k-step kk) from a wave slab
__device__ __forceinline__ bf16x8 slab_frag(const short* slab, int kk, int lane) {
  s8v v = *reinterpret_cast<const s8v*>(slab + (lane & 15) * PLD + kk * 32 + 8 * (lane >> 4));
  return __builtin_bit_cast(bf16x8, v);
}

// A fragment straight from global rows (row-major, k contiguous)
__device__ __forceinline__ bf16x8 gfrag(const bf16_t* rowp, int kk, int lane) {
  return __builtin_bit_cast(bf16x8, *reinterpret_cast<const s8v*>(rowp + kk * 32 + 8 * (lane >> 4)));
}

__device__ __forceinline__ float grp16_max(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float grp16_sum(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

struct AttnArgs {
  const bf16_t* qkv;   // [B*S][3*H*D]
  const bf16_t* out;   // ctx [B*S][H*D] (bwd: O)
  const bf16_t* dout;  // dctx (bwd)
  bf16_t* ctx;         // fwd output
  bf16_t* dqkv;        // bwd output [B*S][3*H*D]
  float* lse;          // [B][H][S] (log2 domain)
  float* dvec;         // [B][H][S] rowsum(dO*O)
  const int* key_len;  // [B] or null
  int B, S, H;
  float scale;
  DropCfg drop;
};

__global__ void __launch_bounds__(256) attn_fwd_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) short Ks[KB * LDT];
  __shared__ __attribute__((aligned(16))) short Vs[KB * LDT];
  __shared__ __attribute__((aligned(16))) short Ps[4][16 * PLD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.z, h = blockIdx.y;
  const int S = a.S, H = a.H, C = H * D;
  const long ldq = 3L * C;
  const int q0 = blockIdx.x * QB + wave * 16;
  int klen = a.key_len ? a.key_len[b] : S;
  klen = klen < 1 ? 1 : (klen > S ? S : klen);
  const bf16_t* base = a.qkv + (long)b * S * ldq;
  const bf16_t* qrow = base + (long)(q0 + (lane & 15)) * ldq + h * D;
  const bf16x8 qf0 = gfrag(qrow, 0, lane), qf1 = gfrag(qrow, 1, lane);
  const float c2 = a.scale * LOG2E;
  const long bh = (long)b * H + h;
  const uint64_t bhss = (uint64_t)bh * S * S;  // dropout index of element (q, key): bhss + q*S + key

  f4v o[4];
  float m[4], l[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) o[t] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    m[r] = -INFINITY;
    l[r] = 0.f;
  }
  short* slab = Ps[wave];
  const int nkb = (klen + KB - 1) / KB;
  for (int kb = 0; kb < nkb; ++kb) {
    const int k0 = kb * KB;
    __syncthreads();
    tile_load(Ks, base + (long)k0 * ldq + C + h * D, ldq, tid);
    tile_load(Vs, base + (long)k0 * ldq + 2 * C + h * D, ldq, tid);
    __syncthreads();
    f4v s[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f4v{0.f, 0.f, 0.f, 0.f};
      s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf0, read_frag<64, true>(Ks, t * 16, 0, lane), s[t], 0, 0, 0);
      s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf1, read_frag<64, true>(Ks, t * 16, 32, lane), s[t], 0, 0, 0);
    }
    float alpha[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int key = k0 + t * 16 + (lane & 15);
        const float v = key < klen ? s[t][r] * c2 : -INFINITY;
        s[t][r] = v;
        mx = fmaxf(mx, v);
      }
      mx = grp16_max(mx);
      const float mn = fmaxf(m[r], mx);
      alpha[r] = exp2f(m[r] - mn);
      m[r] = mn;
      float ls = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float p = exp2f(s[t][r] - mn);
        ls += p;
        s[t][r] = p;
      }
      l[r] = l[r] * alpha[r] + ls;
    }
    if (a.drop.on) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = q0 + (lane >> 4) * 4 + r;
          const int key = k0 + t * 16 + (lane & 15);
          s[t][r] *= drop_mul(a.drop, bhss + (uint32_t)(q * S + key));
        }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[t][r] *= alpha[r];
    slab_store(slab, s, lane);
    __builtin_amdgcn_wave_barrier();
    const bf16x8 p0 = slab_frag(slab, 0, lane), p1 = slab_frag(slab, 1, lane);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      o[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(p0, read_frag<64, false>(Vs, t * 16, 0, lane), o[t], 0, 0, 0);
      o[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(p1, read_frag<64, false>(Vs, t * 16, 32, lane), o[t], 0, 0, 0);
    }
    __builtin_amdgcn_wave_barrier();
  }
  float inv[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float lt = grp16_sum(l[r]);
    inv[r] = 1.f / lt;
    if ((lane & 15) == 0) a.lse[bh * S + q0 + (lane >> 4) * 4 + r] = m[r] + log2f(lt);
  }
  // normalise, stage through the wave slab, 16-B row stores
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) o[t][r] *= inv[r];
  slab_store(slab, o, lane);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = lane + i * 64;  // 16 rows x 8 chunks
    const int r = c >> 3, col = (c & 7) * 8;
    *reinterpret_cast<s8v*>(a.ctx + ((long)b * S + q0 + r) * C + h * D + col) =
        *reinterpret_cast<const s8v*>(slab + r * PLD + col);
  }
}

// Dv[b,h,q] = sum_d dO[q, h*D+d] * O[q, h*D+d]: 8 lanes x 8 elements per (row, head)
__global__ void __launch_bounds__(256) attn_bwd_prep_kernel(AttnArgs a) {
  const long g = (long)blockIdx.x * 32 + (threadIdx.x >> 3);
  const int sub = threadIdx.x & 7;
  const int H = a.H, S = a.S, C = H * D;
  const long rows = (long)a.B * S * H;
  if (g >= rows) return;
  const long row = g / H;  // b*S + q
  const int h = (int)(g - row * H);
  const bf16_t* po = a.out + row * C + h * D + sub * 8;
  const bf16_t* pd = a.dout + row * C + h * D + sub * 8;
  us8 uo = *reinterpret_cast<const us8*>(po), ud = *reinterpret_cast<const us8*>(pd);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += bf2f(uo[j]) * bf2f(ud[j]);
  s += __shfl_xor(s, 1, 64);
  s += __shfl_xor(s, 2, 64);
  s += __shfl_xor(s, 4, 64);
  if (sub == 0) {
    const long b = row / S, q = row - b * S;
    a.dvec[(b * H + h) * S + q] = s;
  }
}

__global__ void __launch_bounds__(256) attn_bwd_dkv_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) short Qs[QB * LDT];
  __shared__ __attribute__((aligned(16))) short Gs[QB * LDT];  // dO
  __shared__ __attribute__((aligned(16))) short Ps[4][16 * PLD];
  __shared__ __attribute__((aligned(16))) short Ds[4][16 * PLD];
  __shared__ float lse_s[QB], dv_s[QB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.z, h = blockIdx.y;
  const int S = a.S, H = a.H, C = H * D;
  const long ldq = 3L * C;
  const int k0 = blockIdx.x * KB + wave * 16;  // this wave's 16 keys
  int klen = a.key_len ? a.key_len[b] : S;
  klen = klen < 1 ? 1 : (klen > S ? S : klen);
  const long bh = (long)b * H + h;
  const uint64_t bhss = (uint64_t)bh * S * S;  // dropout index of element (q, key): bhss + q*S + key
  const bf16_t* base = a.qkv + (long)b * S * ldq;
  const bf16_t* krow = base + (long)(k0 + (lane & 15)) * ldq + C + h * D;
  const bf16_t* vrow = base + (long)(k0 + (lane & 15)) * ldq + 2 * C + h * D;
  const bf16x8 kf0 = gfrag(krow, 0, lane), kf1 = gfrag(krow, 1, lane);
  const bf16x8 vf0 = gfrag(vrow, 0, lane), vf1 = gfrag(vrow, 1, lane);
  const float c2 = a.scale * LOG2E;
  f4v dk[4], dv[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) dk[t] = dv[t] = f4v{0.f, 0.f, 0.f, 0.f};
  short* pslab = Ps[wave];
  short* dslab = Ds[wave];
  const bool any_valid = blockIdx.x * KB < klen;
  const int nqb = any_valid ? S / QB : 0;
  for (int qb = 0; qb < nqb; ++qb) {
    const int q0 = qb * QB;
    __syncthreads();
    tile_load(Qs, base + (long)q0 * ldq + h * D, ldq, tid);
    tile_load(Gs, a.dout + ((long)b * S + q0) * C + h * D, C, tid);
    if (tid < QB) {
      lse_s[tid] = a.lse[bh * S + q0 + tid];
      dv_s[tid] = a.dvec[bh * S + q0 + tid];
    }
    __syncthreads();
    // S^T: rows = keys (this wave), cols = queries
    f4v p[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      p[t] = f4v{0.f, 0.f, 0.f, 0.f};
      p[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf0, read_frag<64, true>(Qs, t * 16, 0, lane), p[t], 0, 0, 0);
      p[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf1, read_frag<64, true>(Qs, t * 16, 32, lane), p[t], 0, 0, 0);
      dp[t] = f4v{0.f, 0.f, 0.f, 0.f};
      dp[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf0, read_frag<64, true>(Gs, t * 16, 0, lane), dp[t], 0, 0, 0);
      dp[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf1, read_frag<64, true>(Gs, t * 16, 32, lane), dp[t], 0, 0, 0);
    }
    f4v pd[4], ds[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int qi = t * 16 + (lane & 15);
      const float ls = lse_s[qi], dvq = dv_s[qi];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = k0 + (lane >> 4) * 4 + r;
        const float pr = key < klen ? exp2f(p[t][r] * c2 - ls) : 0.f;
        const float mul = a.drop.on ? drop_mul(a.drop, bhss + (uint32_t)((q0 + qi) * S + key)) : 1.f;
        pd[t][r] = pr * mul;
        ds[t][r] = pr * (dp[t][r] * mul - dvq);
      }
    }
    slab_store(pslab, pd, lane);
    slab_store(dslab, ds, lane);
    __builtin_amdgcn_wave_barrier();
    const bf16x8 pa0 = slab_frag(pslab, 0, lane), pa1 = slab_frag(pslab, 1, lane);
    const bf16x8 da0 = slab_frag(dslab, 0, lane), da1 = slab_frag(dslab, 1, lane);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      dv[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa0, read_frag<64, false>(Gs, t * 16, 0, lane), dv[t], 0, 0, 0);
      dv[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa1, read_frag<64, false>(Gs, t * 16, 32, lane), dv[t], 0, 0, 0);
      dk[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da0, read_frag<64, false>(Qs, t * 16, 0, lane), dk[t], 0, 0, 0);
      dk[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da1, read_frag<64, false>(Qs, t * 16, 32, lane), dk[t], 0, 0, 0);
    }
    __builtin_amdgcn_wave_barrier();
  }
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) dk[t][r] *= a.scale;
  // stage through the slabs -> 16-B stores into dqkv (K and V thirds)
  slab_store(pslab, dk, lane);
  slab_store(dslab, dv, lane);
  __builtin_amdgcn_wave_barrier();
  bf16_t* drow = a.dqkv + ((long)b * S + k0) * ldq;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = lane + i * 64;
    const int r = c >> 3, col = (c & 7) * 8;
    *reinterpret_cast<s8v*>(drow + (long)r * ldq + C + h * D + col) =
        *reinterpret_cast<const s8v*>(pslab + r * PLD + col);
    *reinterpret_cast<s8v*>(drow + (long)r * ldq + 2 * C + h * D + col) =
        *reinterpret_cast<const s8v*>(dslab + r * PLD + col);
  }
}

__global__ void __launch_bounds__(256) attn_bwd_dq_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) short Ks[KB * LDT];
  __shared__ __attribute__((aligned(16))) short Vs[KB * LDT];
  __shared__ __attribute__((aligned(16))) short Ds[4][16 * PLD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.z, h = blockIdx.y;
  const int S = a.S, H = a.H, C = H * D;
  const long ldq = 3L * C;
  const int q0 = blockIdx.x * QB + wave * 16;
  int klen = a.key_len ? a.key_len[b] : S;
  klen = klen < 1 ? 1 : (klen > S ? S : klen);
  const long bh = (long)b * H + h;
  const uint64_t bhss = (uint64_t)bh * S * S;  // dropout index of element (q, key): bhss + q*S + key
  const bf16_t* base = a.qkv + (long)b * S * ldq;
  const bf16_t* qrow = base + (long)(q0 + (lane & 15)) * ldq + h * D;
  const bf16_t* grow = a.dout + ((long)b * S + q0 + (lane & 15)) * C + h * D;
  const bf16x8 qf0 = gfrag(qrow, 0, lane), qf1 = gfrag(qrow, 1, lane);
  const bf16x8 gf0 = gfrag(grow, 0, lane), gf1 = gfrag(grow, 1, lane);
  const float c2 = a.scale * LOG2E;
  float ls[4], dvq[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = q0 + (lane >> 4) * 4 + r;
    ls[r] = a.lse[bh * S + q];
    dvq[r] = a.dvec[bh * S + q];
  }
  f4v dq[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) dq[t] = f4v{0.f, 0.f, 0.f, 0.f};
  short* dslab = Ds[wave];
  const int nkb = (klen + KB - 1) / KB;
  for (int kb = 0; kb < nkb; ++kb) {
    const int k0 = kb * KB;
    __syncthreads();
    tile_load(Ks, base + (long)k0 * ldq + C + h * D, ldq, tid);
    tile_load(Vs, base + (long)k0 * ldq + 2 * C + h * D, ldq, tid);
    __syncthreads();
    f4v s[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f4v{0.f, 0.f, 0.f, 0.f};
      s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf0, read_frag<64, true>(Ks, t * 16, 0, lane), s[t], 0, 0, 0);
      s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf1, read_frag<64, true>(Ks, t * 16, 32, lane), s[t], 0, 0, 0);
      dp[t] = f4v{0.f, 0.f, 0.f, 0.f};
      dp[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gf0, read_frag<64, true>(Vs, t * 16, 0, lane), dp[t], 0, 0, 0);
      dp[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gf1, read_frag<64, true>(Vs, t * 16, 32, lane), dp[t], 0, 0, 0);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int key = k0 + t * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = q0 + (lane >> 4) * 4 + r;
        const float pr = key < klen ? exp2f(s[t][r] * c2 - ls[r]) : 0.f;
        const float mul = a.drop.on ? drop_mul(a.drop, bhss + (uint32_t)(q * S + key)) : 1.f;
        s[t][r] = pr * (dp[t][r] * mul - dvq[r]);
      }
    }
    slab_store(dslab, s, lane);
    __builtin_amdgcn_wave_barrier();
    const bf16x8 d0 = slab_frag(dslab, 0, lane), d1 = slab_frag(dslab, 1, lane);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      dq[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(d0, read_frag<64, false>(Ks, t * 16, 0, lane), dq[t], 0, 0, 0);
      dq[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(d1, read_frag<64, false>(Ks, t * 16, 32, lane), dq[t], 0, 0, 0);
    }
    __builtin_amdgcn_wave_barrier();
  }
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) dq[t][r] *= a.scale;
  slab_store(dslab, dq, lane);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = lane + i * 64;
    const int r = c >> 3, col = (c & 7) * 8;
    *reinterpret_cast<s8v*>(a.dqkv + ((long)b * S + q0 + r) * ldq + h * D + col) =
        *reinterpret_cast<const s8v*>(dslab + r * PLD + col);
  }
}

// ---------------------------------------------------------------------------
// Fused backward for short sequences (S = 64 or 128, BERT fine-tuning): ONE workgroup per
// (batch, head) holds the whole head in LDS, so the three-kernel path's prep pass, its
// second recomputation of P / dP / the dropout hash (dQ kernel) and its per-block reloads
// of Q / dO / K / V all disappear:
//   load   Q, dO, K -> LDS; this wave's 16 K / V rows -> A fragments; Dv = rowsum(dO * O)
//   A      (wave w = keys 16w..16w+15, all S queries)
//          S^T = K Q^T, dP^T = V dO^T  ->  P, dS = P (dP * mask - Dv)  -> LDS [q][key]
//          dV = P^T dO, dK = dS^T Q    (P^T / dS^T as transposed reads of the [q][key] arrays)
//   B      (wave w = queries 16w..16w+15)  dQ = dS K   (dS rows straight from LDS)
// Every P / dS element is computed (and its dropout bit hashed) once instead of twice.
// LDS: 2 x [S][72] + [S][S + 8] bf16 = 72 KB at S = 128 (two 8-wave blocks per CU; the
// first version kept K, P and dS in separate arrays, 124 KB, one block per CU: 37-38 us).
template <int LD>
__device__ __forceinline__ bf16x8 frag_kc(const short* lds, int r0, int k0, int lane) {
  s8v v = *reinterpret_cast<const s8v*>(lds + (r0 + (lane & 15)) * LD + k0 + 8 * (lane >> 4));
  return __builtin_bit_cast(bf16x8, v);
}
// element (r, k) at lds[k * LD + r] (r contiguous): the transposed read
template <int LD>
__device__ __forceinline__ bf16x8 frag_nc(const short* lds, int r0, int k0, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const short* b0 = lds + (k0 + 8 * g + q) * LD + r0 + 4 * p;
  s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(b0));
  s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(b0 + 4 * LD));
  s8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// C-layout 16 x 64 fp32 (4 column tiles, lane l: row 4 (l >> 4) + r, column 16 t + (l & 15))
// -> bf16 [16][LDT] slab, then 16-B row stores to dst rows (pitch ld)
__device__ __forceinline__ void stage_store(short* slab, const f4v (&v)[4], bf16_t* dst, long ld, int lane) {
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) slab[((lane >> 4) * 4 + r) * LDT + t * 16 + (lane & 15)] = (short)f2bf(v[t][r]);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = lane + i * 64;
    const int r = c >> 3, col = (c & 7) * 8;
    *reinterpret_cast<s8v*>(dst + (long)r * ld + col) = *reinterpret_cast<const s8v*>(slab + r * LDT + col);
  }
}

template <int SQ>
__global__ void __launch_bounds__(SQ * 4) __attribute__((amdgpu_waves_per_eu(4))) attn_bwd_fused_kernel(AttnArgs a) {
  constexpr int NW = SQ / 16, NT = NW * 64, TQ = SQ / 16, PL = SQ + 8, LCH = SQ * 8 / NT;
  // Qs: Q; Gs: dO (phase A), then K (phase B); Xs [q][key]: each wave's P columns, then
  // its dS columns (P is dead once dV is accumulated).  72 KB at S = 128: two blocks per CU.
  __shared__ __attribute__((aligned(16))) short Qs[SQ * LDT];
  __shared__ __attribute__((aligned(16))) short Gs[SQ * LDT];
  __shared__ __attribute__((aligned(16))) short Xs[SQ * PL];
  __shared__ float lse_s[SQ], dv_s[SQ];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bh = blockIdx.x;
  const int b = bh / a.H, h = bh - b * a.H;
  const int H = a.H, C = H * D;
  const long ldq = 3L * C;
  int klen = a.key_len ? a.key_len[b] : SQ;
  klen = klen < 1 ? 1 : (klen > SQ ? SQ : klen);
  const uint64_t bhss = (uint64_t)bh * SQ * SQ;
  const bf16_t* base = a.qkv + (long)b * SQ * ldq;
  const bf16_t* gbase = a.dout + (long)b * SQ * C + h * D;
  const bf16_t* obase = a.out + (long)b * SQ * C + h * D;

  // ---- loads: Q / dO tiles, Dv = rowsum(dO * O)
#pragma unroll
  for (int i = 0; i < LCH; ++i) {
    const int c = tid + i * NT;
    const int r = c >> 3, col = (c & 7) * 8;
    const s8v qv = *reinterpret_cast<const s8v*>(base + (long)r * ldq + h * D + col);
    const us8 gv = *reinterpret_cast<const us8*>(gbase + (long)r * C + col);
    const us8 ov = *reinterpret_cast<const us8*>(obase + (long)r * C + col);
    *reinterpret_cast<s8v*>(Qs + r * LDT + col) = qv;
    *reinterpret_cast<us8*>(Gs + r * LDT + col) = gv;
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += bf2f(gv[j]) * bf2f(ov[j]);
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    s += __shfl_xor(s, 4, 64);
    if ((c & 7) == 0) dv_s[r] = s;
  }
  if (tid < SQ) lse_s[tid] = a.lse[(long)bh * SQ + tid];
  const int k0 = wave * 16;
  const bf16_t* krow = base + (long)(k0 + (lane & 15)) * ldq + C + h * D;
  const bf16_t* vrow = krow + C;
  const bf16x8 kf0 = gfrag(krow, 0, lane), kf1 = gfrag(krow, 1, lane);
  const bf16x8 vf0 = gfrag(vrow, 0, lane), vf1 = gfrag(vrow, 1, lane);
  const float c2 = a.scale * LOG2E;
  __syncthreads();

  // ---- phase A: this wave's 16 keys against all queries
  s4v dsr[TQ];  // this wave's dS^T values, held until P's columns are consumed
  {
    f4v p[TQ], dp[TQ];
#pragma unroll
    for (int t = 0; t < TQ; ++t) {
      p[t] = f4v{0.f, 0.f, 0.f, 0.f};
      p[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf0, frag_kc<LDT>(Qs, t * 16, 0, lane), p[t], 0, 0, 0);
      p[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf1, frag_kc<LDT>(Qs, t * 16, 32, lane), p[t], 0, 0, 0);
      dp[t] = f4v{0.f, 0.f, 0.f, 0.f};
      dp[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf0, frag_kc<LDT>(Gs, t * 16, 0, lane), dp[t], 0, 0, 0);
      dp[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf1, frag_kc<LDT>(Gs, t * 16, 32, lane), dp[t], 0, 0, 0);
    }
    // p[t][r] = S^T[key = k0 + 4 (l >> 4) + r][q = 16 t + (l & 15)]
    const int kr = k0 + (lane >> 4) * 4;
#pragma unroll
    for (int t = 0; t < TQ; ++t) {
      const int qi = t * 16 + (lane & 15);
      const float ls = lse_s[qi], dvq = dv_s[qi];
      s4v pk;
      float dm[4] = {1.f, 1.f, 1.f, 1.f};  // the row's four consecutive keys: two hashes
      if (a.drop.on) drop_mul4(a.drop, bhss + (uint32_t)(qi * SQ + kr), dm);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kr + r;
        const float pr = key < klen ? exp2f(p[t][r] * c2 - ls) : 0.f;
        const float mul = dm[r];
        pk[r] = (short)f2bf(pr * mul);
        dsr[t][r] = (short)f2bf(pr * (dp[t][r] * mul - dvq));
      }
      *reinterpret_cast<s4v*>(Xs + qi * PL + kr) = pk;
    }
  }
  f4v dk[4], dv[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) dk[t] = dv[t] = f4v{0.f, 0.f, 0.f, 0.f};
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int kk = 0; kk < SQ / 32; ++kk) {
    const bf16x8 pa = frag_nc<PL>(Xs, k0, kk * 32, lane);  // P^T: row = key, k = query
#pragma unroll
    for (int t = 0; t < 4; ++t)
      dv[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, frag_nc<LDT>(Gs, t * 16, kk * 32, lane), dv[t], 0, 0, 0);
  }
  // P's columns of this wave are read: overwrite them with dS
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  {
    const int kr = k0 + (lane >> 4) * 4;
#pragma unroll
    for (int t = 0; t < TQ; ++t) *reinterpret_cast<s4v*>(Xs + (t * 16 + (lane & 15)) * PL + kr) = dsr[t];
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int kk = 0; kk < SQ / 32; ++kk) {
    const bf16x8 da = frag_nc<PL>(Xs, k0, kk * 32, lane);  // dS^T
#pragma unroll
    for (int t = 0; t < 4; ++t)
      dk[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da, frag_nc<LDT>(Qs, t * 16, kk * 32, lane), dk[t], 0, 0, 0);
  }
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) dk[t][r] *= a.scale;
  __syncthreads();  // every wave's dS columns written; dO no longer read

  // K into the dO region (its load latency is covered by the CU's other block)
#pragma unroll
  for (int i = 0; i < LCH; ++i) {
    const int c = tid + i * NT;
    const int r = c >> 3, col = (c & 7) * 8;
    *reinterpret_cast<s8v*>(Gs + r * LDT + col) = *reinterpret_cast<const s8v*>(base + (long)r * ldq + C + h * D + col);
  }
  __syncthreads();

  // ---- phase B: dQ for this wave's 16 queries
  const int q0 = wave * 16;
  f4v dq[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) dq[t] = f4v{0.f, 0.f, 0.f, 0.f};
  const int nkk = (klen + 31) / 32;
  for (int kk = 0; kk < nkk; ++kk) {
    const bf16x8 da = frag_kc<PL>(Xs, q0, kk * 32, lane);  // dS: row = query, k = key
#pragma unroll
    for (int t = 0; t < 4; ++t)
      dq[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da, frag_nc<LDT>(Gs, t * 16, kk * 32, lane), dq[t], 0, 0, 0);
  }
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) dq[t][r] *= a.scale;
  __syncthreads();  // dS and K no longer read: every region is staging space now

  bf16_t* drow = a.dqkv + ((long)b * SQ + k0) * ldq + h * D;
  stage_store(Qs + wave * 16 * LDT, dk, drow + C, ldq, lane);
  stage_store(Gs + wave * 16 * LDT, dv, drow + 2 * C, ldq, lane);
  stage_store(Xs + wave * 16 * LDT, dq, a.dqkv + ((long)b * SQ + q0) * ldq + h * D, ldq, lane);
}

// Forward for S = 64 / 128: one workgroup per (batch, head), all S keys' K and V issued
// to LDS up front (one memory round trip instead of one per 64-key block), then each
// wave's 16 query rows take an exact (not online) softmax over the whole key row.
// LDS: 2 x [S][72] = 36 KB at S = 128.  Once every wave holds its scores in registers the
// K image is dead, and each wave stages its P (64 keys at a time, [16][72]) and finally its
// output tile in its own 16 rows of it -- three 8-wave blocks per CU (72 VGPRs), so the
// B x H = 768 blocks of BERT-base b64 run in one round instead of 1.5 (per-wave P slabs
// beside K / V took 72 KB: two blocks per CU).
template <int SQ>
__global__ void __launch_bounds__(SQ * 4) attn_fwd_short_kernel(AttnArgs a) {
  constexpr int NW = SQ / 16, NT = NW * 64, TK = SQ / 16;
  static_assert(NW * 16 == SQ, "one 16-row slab of the K image per wave");
  __shared__ __attribute__((aligned(16))) short Ks[SQ * LDT];
  __shared__ __attribute__((aligned(16))) short Vs[SQ * LDT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bh = blockIdx.x;
  const int b = bh / a.H, h = bh - b * a.H;
  const int C = a.H * D;
  const long ldq = 3L * C;
  int klen = a.key_len ? a.key_len[b] : SQ;
  klen = klen < 1 ? 1 : (klen > SQ ? SQ : klen);
  const uint64_t bhss = (uint64_t)bh * SQ * SQ;
  const bf16_t* base = a.qkv + (long)b * SQ * ldq;
#pragma unroll
  for (int i = 0; i < SQ * 8 / NT; ++i) {
    const int c = tid + i * NT;
    const int r = c >> 3, col = (c & 7) * 8;
    const s8v kv = *reinterpret_cast<const s8v*>(base + (long)r * ldq + C + h * D + col);
    const s8v vv = *reinterpret_cast<const s8v*>(base + (long)r * ldq + 2 * C + h * D + col);
    *reinterpret_cast<s8v*>(Ks + r * LDT + col) = kv;
    *reinterpret_cast<s8v*>(Vs + r * LDT + col) = vv;
  }
  const int q0 = wave * 16;
  const bf16_t* qrow = base + (long)(q0 + (lane & 15)) * ldq + h * D;
  const bf16x8 qf0 = gfrag(qrow, 0, lane), qf1 = gfrag(qrow, 1, lane);
  const float c2 = a.scale * LOG2E;
  __syncthreads();
  // s[t][r] = S[q = q0 + 4 (l >> 4) + r][key = 16 t + (l & 15)]
  f4v s[TK];
#pragma unroll
  for (int t = 0; t < TK; ++t) {
    s[t] = f4v{0.f, 0.f, 0.f, 0.f};
    s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf0, frag_kc<LDT>(Ks, t * 16, 0, lane), s[t], 0, 0, 0);
    s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf1, frag_kc<LDT>(Ks, t * 16, 32, lane), s[t], 0, 0, 0);
  }
  float m[4], l[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < TK; ++t) {
      const int key = t * 16 + (lane & 15);
      const float v = key < klen ? s[t][r] * c2 : -INFINITY;
      s[t][r] = v;
      mx = fmaxf(mx, v);
    }
    m[r] = grp16_max(mx);
    float ls = 0.f;
#pragma unroll
    for (int t = 0; t < TK; ++t) {
      const float p = exp2f(s[t][r] - m[r]);
      ls += p;
      s[t][r] = p;
    }
    l[r] = grp16_sum(ls);
  }
  // every wave's QK^T reads of Ks are done past this barrier: its rows become P slabs
  __syncthreads();
  short* slab = Ks + wave * 16 * LDT;
  f4v o[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) o[t] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int half = 0; half < SQ / 64; ++half) {
    if (half) __builtin_amdgcn_wave_barrier();  // the previous half's P reads precede these writes
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      const int t = half * 4 + tt;
      // keys across lanes: a lane pair shares each row's hash (drop_mul_lanepair; SQ is even)
      float dm[4] = {1.f, 1.f, 1.f, 1.f};
      if (a.drop.on) {
        static_assert(SQ % 2 == 0, "lane-pair dropout hashing needs an even row length");
        const int keyev = t * 16 + (lane & 14);
#pragma unroll
        for (int rr = 0; rr < 4; rr += 2) {
          const int qh = q0 + (lane >> 4) * 4 + rr + (lane & 1);
          drop_mul_lanepair(a.drop, (bhss + (uint32_t)(qh * SQ + keyev)) >> 1, lane, dm[rr], dm[rr + 1]);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
        slab[((lane >> 4) * 4 + r) * LDT + tt * 16 + (lane & 15)] = (short)f2bf(s[t][r] * dm[r]);
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      const bf16x8 pf = frag_kc<LDT>(slab, 0, k2 * 32, lane);
      const int kk = half * 2 + k2;
#pragma unroll
      for (int t = 0; t < 4; ++t)
        o[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf, frag_nc<LDT>(Vs, t * 16, kk * 32, lane), o[t], 0, 0, 0);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float inv = 1.f / l[r];
    if ((lane & 15) == 0) a.lse[(long)bh * SQ + q0 + (lane >> 4) * 4 + r] = m[r] + log2f(l[r]);
#pragma unroll
    for (int t = 0; t < 4; ++t) o[t][r] *= inv;
  }
  __builtin_amdgcn_wave_barrier();
  stage_store(slab, o, a.ctx + ((long)b * SQ + q0) * C + h * D, C, lane);
}

bool shape_ok(int S, int H) { return S > 0 && S % 64 == 0 && H > 0; }

// CLOUD_AMD_ATTN_FUSED_BWD=0 keeps the three-kernel backward at S <= 128 (A/B runs)
bool fused_bwd_enabled() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CLOUD_AMD_ATTN_FUSED_BWD");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v != 0;
}

}  // namespace

extern "C" {

// ctx = softmax(Q K^T * scale + keymask) (dropout) V ; lse[B][H][S] saved for the backward.
int ca_attn_fwd(const bf16_t* qkv, bf16_t* ctx, float* lse, const int* key_len, int B, int S, int H, float scale,
                float p_drop, uint64_t seed, hipStream_t s) {
  if (!shape_ok(S, H)) return -1;
  AttnArgs a{};
  a.qkv = qkv; a.ctx = ctx; a.lse = lse; a.key_len = key_len;
  a.B = B; a.S = S; a.H = H; a.scale = scale; a.drop = make_drop(p_drop, seed);
  if ((S == 64 || S == 128) && fused_bwd_enabled()) {
    if (S == 128) attn_fwd_short_kernel<128><<<B * H, 512, 0, s>>>(a);
    else attn_fwd_short_kernel<64><<<B * H, 256, 0, s>>>(a);
    CA_LAUNCH_CHECK();
    return 0;
  }
  attn_fwd_kernel<<<dim3(S / QB, H, B), 256, 0, s>>>(a);
  CA_LAUNCH_CHECK();
  return 0;
}

// dqkv (all three thirds written) from dctx; dvec: [B][H][S] fp32 scratch.
int ca_attn_bwd(const bf16_t* qkv, const bf16_t* out, const bf16_t* dout, const float* lse, float* dvec,
                bf16_t* dqkv, const int* key_len, int B, int S, int H, float scale, float p_drop, uint64_t seed,
                hipStream_t s) {
  if (!shape_ok(S, H)) return -1;
  AttnArgs a{};
  a.qkv = qkv; a.out = out; a.dout = dout; a.lse = const_cast<float*>(lse); a.dvec = dvec; a.dqkv = dqkv;
  a.key_len = key_len; a.B = B; a.S = S; a.H = H; a.scale = scale; a.drop = make_drop(p_drop, seed);
  if ((S == 64 || S == 128) && fused_bwd_enabled()) {
    if (S == 128) attn_bwd_fused_kernel<128><<<B * H, 512, 0, s>>>(a);
    else attn_bwd_fused_kernel<64><<<B * H, 256, 0, s>>>(a);
    CA_LAUNCH_CHECK();
    return 0;
  }
  const long rows = (long)B * S * H;
  attn_bwd_prep_kernel<<<ca_cdiv(rows, 32), 256, 0, s>>>(a);
  CA_LAUNCH_CHECK();
  attn_bwd_dkv_kernel<<<dim3(S / KB, H, B), 256, 0, s>>>(a);
  CA_LAUNCH_CHECK();
  attn_bwd_dq_kernel<<<dim3(S / QB, H, B), 256, 0, s>>>(a);
  CA_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
