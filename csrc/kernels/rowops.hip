// Row-wise kernels of the transformer path (K13 / K8 / K14 in SURVEY.md 2.7):
//
//  * LayerNorm forward with the residual add and BOTH dropouts fused:
//        h = res + drop_in(x);   y = drop_out(LN(h) * gamma + beta)
//    one wave per row (C <= 2048, 4 bf16 per lane per step), fp32 statistics;
//  * LayerNorm backward: dh (= the residual-branch gradient) and, when the input
//    was dropped, dx = drop_in'(dh), plus per-block dgamma/dbeta partials
//    reduced deterministically and ACCUMULATED into the (arena) fp32 grads;
//  * column sums of a bf16 matrix (bias gradients) into fp32, accumulated;
//  * token + position + segment embedding gather/sum and its scatter-add
//    backward (fp32 tables and grads, hardware fp32 atomics);
//  * standalone dropout fwd/bwd and a mask materialiser for tests.
// Dropout masks come from the stateless hash of ca_rng.h (never stored).
#include "ca_common.h"
#include "ca_mfma_core.h"
#include "ca_rng.h"


namespace {

typedef unsigned short us4v __attribute__((ext_vector_type(4)));

constexpr int LN_BLK = 256;  // 4 rows (waves) per block

__device__ __forceinline__ void load4(const bf16_t* p, float* v) {
  us4v u = *reinterpret_cast<const us4v*>(p);
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = bf2f(u[j]);
}
__device__ __forceinline__ void store4(bf16_t* p, const float* v) {
  us4v u;
#pragma unroll
  for (int j = 0; j < 4; ++j) u[j] = f2bf(v[j]);
  *reinterpret_cast<us4v*>(p) = u;
}

template <int NV>
__global__ void __launch_bounds__(LN_BLK) ln_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                        const float* __restrict__ gamma, const float* __restrict__ beta,
                                                        bf16_t* __restrict__ y, bf16_t* __restrict__ h_out,
                                                        float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                        long M, int C, float eps, DropCfg din, DropCfg dout,
                                                        const float* __restrict__ xbias) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * (LN_BLK / 64) + (threadIdx.x >> 6);
  if (row >= M) return;
  const int C4 = C >> 2;
  const long base = row * C;
  float v[NV][4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c4 = lane + 64 * i;
    if (c4 < C4) {
      load4(x + base + 4 * c4, v[i]);
      if (xbias) {  // the producing GEMM's bias, applied here instead of in its epilogue
        const f4 xb = *reinterpret_cast<const f4*>(xbias + 4 * c4);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[i][j] += xb[j];
      }
      if (din.on) {
        float m[4];
        drop_mul4(din, base + 4 * c4, m);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[i][j] *= m[j];
      }
      if (res) {
        float r[4];
        load4(res + base + 4 * c4, r);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[i][j] += r[j];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) s += v[i][j];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[i][j] = 0.f;
    }
  }
  const float mean = wave_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
    if (lane + 64 * i < C4) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = v[i][j] - mean;
        q += d * d;
      }
    }
  const float rstd = rsqrtf(wave_sum(q) / (float)C + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c4 = lane + 64 * i;
    if (c4 >= C4) continue;
    if (h_out) store4(h_out + base + 4 * c4, v[i]);
    const f4 g = *reinterpret_cast<const f4*>(gamma + 4 * c4);
    const f4 b = *reinterpret_cast<const f4*>(beta + 4 * c4);
    float o[4], m[4] = {1.f, 1.f, 1.f, 1.f};
    if (dout.on) drop_mul4(dout, base + 4 * c4, m);
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = (v[i][j] - mean) * rstd * g[j] + b[j];
    if (dout.on) {
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] *= m[j];
    }
    store4(y + base + 4 * c4, o);
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// grid-stride over rows; per-block [2][C] partials (dgamma, dbeta) in `part`.
template <int NV>
__global__ void __launch_bounds__(LN_BLK) ln_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ h,
                                                        const float* __restrict__ mean, const float* __restrict__ rstd,
                                                        const float* __restrict__ gamma, bf16_t* __restrict__ dh,
                                                        bf16_t* __restrict__ dx, float* __restrict__ part, long M,
                                                        int C, DropCfg din, DropCfg dout) {
  extern __shared__ float red[];  // [4 waves][3][C]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int C4 = C >> 2;
  // ag / ab: dgamma / dbeta partials; ax: column sums of the gradient this LN hands on
  // (dx after the input dropout, else dh) -- the bias gradient of the dense layer whose
  // output fed the LN (BERT: bo, b2), so no separate column-sum pass re-reads it
  float ag[NV][4], ab[NV][4], ax[NV][4], g[NV][4];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c4 = lane + 64 * i;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      ag[i][j] = ab[i][j] = ax[i][j] = 0.f;
      g[i][j] = c4 < C4 ? gamma[4 * c4 + j] : 0.f;
    }
  }
  const float invC = 1.f / (float)C;
  // software-pipelined over this wave's rows: the next row's dy / h / statistics are in
  // flight while the current row is reduced and stored
  const long stride = (long)gridDim.x * 4;
  long row = (long)blockIdx.x * 4 + wave;
  float nd[NV][4], nx[NV][4], nmu = 0.f, nrs = 0.f;
  auto fetch = [&](long r) {
    if (r >= M) return;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c4 = lane + 64 * i;
      if (c4 < C4) {
        load4(dy + r * C + 4 * c4, nd[i]);
        load4(h + r * C + 4 * c4, nx[i]);
      }
    }
    nmu = mean[r];
    nrs = rstd[r];
  };
  fetch(row);
  for (; row < M; row += stride) {
    const long base = row * C;
    const float mu = nmu, rs = nrs;
    float d[NV][4], xh[NV][4];
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        d[i][j] = nd[i][j];
        xh[i][j] = nx[i][j];
      }
    fetch(row + stride);
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c4 = lane + 64 * i;
      if (c4 < C4) {
        if (dout.on) {
          float m[4];
          drop_mul4(dout, base + 4 * c4, m);
#pragma unroll
          for (int j = 0; j < 4; ++j) d[i][j] *= m[j];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          xh[i][j] = (xh[i][j] - mu) * rs;
          ag[i][j] += d[i][j] * xh[i][j];
          ab[i][j] += d[i][j];
          const float gd = g[i][j] * d[i][j];
          sa += gd;
          sb += gd * xh[i][j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) d[i][j] = xh[i][j] = 0.f;
      }
    }
    const float a = wave_sum(sa) * invC, b = wave_sum(sb) * invC;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c4 = lane + 64 * i;
      if (c4 >= C4) continue;
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = rs * (g[i][j] * d[i][j] - a - xh[i][j] * b);
      store4(dh + base + 4 * c4, o);
      if (dx) {
        if (din.on) {
          float m[4];
          drop_mul4(din, base + 4 * c4, m);
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] *= m[j];
        }
        store4(dx + base + 4 * c4, o);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) ax[i][j] += o[j];
    }
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c4 = lane + 64 * i;
    if (c4 < C4) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        red[(wave * 3 + 0) * C + 4 * c4 + j] = ag[i][j];
        red[(wave * 3 + 1) * C + 4 * c4 + j] = ab[i][j];
        red[(wave * 3 + 2) * C + 4 * c4 + j] = ax[i][j];
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 3 * C; c += LN_BLK) {
    const int k = c / C, col = c - k * C;
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) t += red[(w * 3 + k) * C + col];
    part[(long)blockIdx.x * 3 * C + c] = t;
  }
}

// 16-wave form: the same per-row math with one row per wave (8,192 waves at BERT's M = 8192
// instead of 2,048 walking four rows each: the row's loads, two wave reductions and stores are
// one latency chain, so more waves in flight is the lever), and the block's 16 partial rows
// summed in LDS by a fixed pairing tree (8+8, 4+4, 2+2, 1+1: deterministic) into the same ONE
// [3][C] partial row per block as ln_bwd_kernel -- the finalisation is unchanged.
template <int NV>
__global__ void __launch_bounds__(1024) ln_bwd16_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ h,
                                                        const float* __restrict__ mean, const float* __restrict__ rstd,
                                                        const float* __restrict__ gamma, bf16_t* __restrict__ dh,
                                                        bf16_t* __restrict__ dx, float* __restrict__ part, long M,
                                                        int C, DropCfg din, DropCfg dout) {
  extern __shared__ float red[];  // [8 waves][3][C] partial rows, then gamma [C]
  float* sg = red + 24 * C;       // (gamma from LDS per row: 12 fewer registers per lane)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int C4 = C >> 2;
  for (int c = threadIdx.x; c < C; c += 1024) sg[c] = gamma[c];
  __syncthreads();
  float ag[NV][4], ab[NV][4], ax[NV][4];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) ag[i][j] = ab[i][j] = ax[i][j] = 0.f;
  const float invC = 1.f / (float)C;
  for (long row = (long)blockIdx.x * 16 + wave; row < M; row += (long)gridDim.x * 16) {
    const long base = row * C;
    const float mu = mean[row], rs = rstd[row];
    float d[NV][4], xh[NV][4];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c4 = lane + 64 * i;
      if (c4 < C4) {
        load4(dy + base + 4 * c4, d[i]);
        load4(h + base + 4 * c4, xh[i]);
      }
    }
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c4 = lane + 64 * i;
      if (c4 < C4) {
        const f4 gv = *reinterpret_cast<const f4*>(sg + 4 * c4);
        if (dout.on) {
          float m[4];
          drop_mul4(dout, base + 4 * c4, m);
#pragma unroll
          for (int j = 0; j < 4; ++j) d[i][j] *= m[j];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          xh[i][j] = (xh[i][j] - mu) * rs;
          ag[i][j] += d[i][j] * xh[i][j];
          ab[i][j] += d[i][j];
          const float gd = gv[j] * d[i][j];
          sa += gd;
          sb += gd * xh[i][j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) d[i][j] = xh[i][j] = 0.f;
      }
    }
    const float a = wave_sum(sa) * invC, b = wave_sum(sb) * invC;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c4 = lane + 64 * i;
      if (c4 >= C4) continue;
      const f4 gv = *reinterpret_cast<const f4*>(sg + 4 * c4);
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = rs * (gv[j] * d[i][j] - a - xh[i][j] * b);
      store4(dh + base + 4 * c4, o);
      if (dx) {
        if (din.on) {
          float m[4];
          drop_mul4(din, base + 4 * c4, m);
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] *= m[j];
        }
        store4(dx + base + 4 * c4, o);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) ax[i][j] += o[j];
    }
  }
  // fixed pairing tree over the 16 waves' partials
#pragma unroll
  for (int sp = 8; sp >= 1; sp >>= 1) {
    if (wave >= sp && wave < 2 * sp) {
      float* r = red + (long)(wave - sp) * 3 * C;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c4 = lane + 64 * i;
        if (c4 < C4) {
          *reinterpret_cast<f4*>(r + 4 * c4) = f4{ag[i][0], ag[i][1], ag[i][2], ag[i][3]};
          *reinterpret_cast<f4*>(r + C + 4 * c4) = f4{ab[i][0], ab[i][1], ab[i][2], ab[i][3]};
          *reinterpret_cast<f4*>(r + 2 * C + 4 * c4) = f4{ax[i][0], ax[i][1], ax[i][2], ax[i][3]};
        }
      }
    }
    __syncthreads();
    if (wave < sp) {
      const float* r = red + (long)wave * 3 * C;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c4 = lane + 64 * i;
        if (c4 < C4) {
          const f4 p0 = *reinterpret_cast<const f4*>(r + 4 * c4);
          const f4 p1 = *reinterpret_cast<const f4*>(r + C + 4 * c4);
          const f4 p2 = *reinterpret_cast<const f4*>(r + 2 * C + 4 * c4);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            ag[i][j] += p0[j];
            ab[i][j] += p1[j];
            ax[i][j] += p2[j];
          }
        }
      }
    }
    __syncthreads();
  }
  if (wave == 0) {
    float* dst = part + (long)blockIdx.x * 3 * C;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c4 = lane + 64 * i;
      if (c4 < C4) {
        *reinterpret_cast<f4*>(dst + 4 * c4) = f4{ag[i][0], ag[i][1], ag[i][2], ag[i][3]};
        *reinterpret_cast<f4*>(dst + C + 4 * c4) = f4{ab[i][0], ab[i][1], ab[i][2], ab[i][3]};
        *reinterpret_cast<f4*>(dst + 2 * C + 4 * c4) = f4{ax[i][0], ax[i][1], ax[i][2], ax[i][3]};
      }
    }
  }
}

// out[c] (+)= sum_p part[p*stride + c], for c < N; out2 / out3 (optional) get columns
// N..2N-1 / 2N..3N-1.  Block = 16 columns x 16 part-lanes (enough waves in flight to
// hide the partial-slab reads; deterministic fixed-order tree).
__global__ void __launch_bounds__(256) col_finalize_kernel(const float* __restrict__ part, int nparts, long stride,
                                                           int N, float* __restrict__ out, float* __restrict__ out2,
                                                           int accumulate, float* __restrict__ out3 = nullptr) {
  __shared__ float red[16][17];
  const int cl = threadIdx.x & 15, pl = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  const int total = out3 ? 3 * N : (out2 ? 2 * N : N);
  float t = 0.f;
  if (c < total) {
#pragma unroll 4
    for (int p = pl; p < nparts; p += 16) t += part[(long)p * stride + c];
  }
  red[pl][cl] = t;
  __syncthreads();
  if (pl != 0 || c >= total) return;
  t = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) t += red[k][cl];
  const int k = c / N;
  float* dst = k == 0 ? out : (k == 1 ? out2 : out3);
  if (!dst) return;
  float* o = dst + (c - k * N);
  *o = accumulate ? *o + t : t;
}

// per-block column partial sums of bf16 X[M][N] (N % 8 == 0): block = 32 col-groups(8 cols) x 8 row lanes
__global__ void __launch_bounds__(256) colsum_part_kernel(const bf16_t* __restrict__ x, long M, int N, long ld,
                                                          float* __restrict__ part, float* __restrict__ fin = nullptr,
                                                          int fin_acc = 0) {
  __shared__ float red[8][256];
  const int cg = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int c0 = (blockIdx.x * 32 + cg) * 8;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < N) {
    for (long r = (long)blockIdx.y * 8 + rl; r < M; r += (long)gridDim.y * 8) {
      us8 u = *reinterpret_cast<const us8*>(x + r * ld + c0);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += bf2f(u[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rl][cg * 8 + j] = acc[j];
  __syncthreads();
  const int c = threadIdx.x;  // 256 columns of this block
  const int gc = blockIdx.x * 256 + c;
  if (gc < N) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += red[k][c];
    if (fin) {  // one row-part (gridDim.y == 1): this is the column sum itself
      fin[gc] = fin_acc ? fin[gc] + t : t;
    } else {
      part[(long)blockIdx.y * N + gc] = t;
    }
  }
}

// h[m] = word[id[m]] + pos[m % S] + type[tt[m]]   (fp32 tables, bf16 out), one wave per row.
__global__ void __launch_bounds__(256) embed_sum_kernel(const int32_t* __restrict__ ids, const int32_t* __restrict__ tts,
                                                        const float* __restrict__ word, const float* __restrict__ pos,
                                                        const float* __restrict__ type, bf16_t* __restrict__ h,
                                                        long M, int S, int C, int pos_offset) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const float* w = word + (long)ids[row] * C;
  const float* p = pos + (long)(row % S + pos_offset) * C;
  const float* t = type ? type + (long)(tts ? tts[row] : 0) * C : nullptr;
  for (int c4 = lane; c4 < C / 4; c4 += 64) {
    f4 a = *reinterpret_cast<const f4*>(w + 4 * c4) + *reinterpret_cast<const f4*>(p + 4 * c4);
    if (t) a += *reinterpret_cast<const f4*>(t + 4 * c4);
    float o[4] = {a[0], a[1], a[2], a[3]};
    store4(h + row * C + 4 * c4, o);
  }
}

// scatter-add backward of embed_sum for the token-type table (and, when the owner kernel
// below cannot take them, word rows): fp32 atomics, skipping the padding id (its row gets
// no gradient, as nn.Embedding(padding_idx) / BERT); the segment table (<= 2 rows in BERT)
// is pre-reduced per wave first.  Each wave takes EB_RW consecutive rows and issues all
// their loads before adding (one memory round trip per column group, not one per row:
// 111 -> a few us at 8192 x 768).
constexpr int EB_RW = 16;
//
// tws / ticket (token types, T <= 2): DETERMINISTIC form -- each block writes its pre-reduced
// [2][C] row into tws[blockIdx.x] instead of adding it atomically, and the block that arrives
// last (agent-scope ticket, as bn.hip group_finalize_kernel) adds the rows in block order.
__global__ void __launch_bounds__(256) embed_bwd_kernel(const bf16_t* __restrict__ dh, const int32_t* __restrict__ ids,
                                                        const int32_t* __restrict__ tts, float* __restrict__ dword,
                                                        float* __restrict__ dtype, long M, int C, int T, int pad_id,
                                                        float* __restrict__ tws, unsigned* __restrict__ ticket) {
  const int lane = threadIdx.x & 63;
  const long wave = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long nw = (long)gridDim.x * 4;
  // uniform trip count for every lane (the block barriers below); lanes past C / 4 idle
  for (int cb = 0; cb < C / 4; cb += 64) {
    const int c4 = cb + lane < C / 4 ? cb + lane : C / 4 - 1;
    const bool cok = cb + lane < C / 4;
    float t0[4] = {0.f, 0.f, 0.f, 0.f}, t1[4] = {0.f, 0.f, 0.f, 0.f};
    for (long row0 = wave * EB_RW; row0 < M; row0 += nw * EB_RW) {
      float g[EB_RW][4];
      int tt[EB_RW];
#pragma unroll
      for (int u = 0; u < EB_RW; ++u) {
        const long row = row0 + u < M ? row0 + u : M - 1;
        load4(dh + row * C + 4 * c4, g[u]);
        tt[u] = (row0 + u < M && cok) ? (tts ? tts[row] : 0) : -1;
      }
#pragma unroll
      for (int u = 0; u < EB_RW; ++u) {
        if (tt[u] < 0) continue;
        const long row = row0 + u;
        if (dword) {
          const int id = ids[row];
          if (id != pad_id) {
            float* w = dword + (long)id * C + 4 * c4;
#pragma unroll
            for (int j = 0; j < 4; ++j) atomicAdd(w + j, g[u][j]);
          }
        }
        if (dtype) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (T <= 2) {
              if (tt[u] == 0) t0[j] += g[u][j];
              else t1[j] += g[u][j];
            } else {
              atomicAdd(dtype + (long)tt[u] * C + 4 * c4 + j, g[u][j]);
            }
          }
        }
      }
    }
    if (dtype && T <= 2) {
      // the block's 4 waves pre-reduce through LDS: one atomic per (block, column) --
      // per-wave atomics put 512 adds on each of the 2 x C addresses (97 us at 8192 x 768)
      __shared__ float tred[4][2][256];
      const int w = threadIdx.x >> 6;
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        tred[w][0][lane * 4 + j] = t0[j];
        tred[w][1][lane * 4 + j] = t1[j];
      }
      __syncthreads();
      for (int k = threadIdx.x; k < 2 * 256; k += 256) {
        const int t = k >> 8, e = k & 255;  // e = lane * 4 + j
        if (t >= T || cb + (e >> 2) >= C / 4) continue;
        const float v = tred[0][t][e] + tred[1][t][e] + tred[2][t][e] + tred[3][t][e];
        const long col = 4 * (cb + (e >> 2)) + (e & 3);
        if (tws) tws[((long)blockIdx.x * 2 + t) * C + col] = v;
        else atomicAdd(dtype + (long)t * C + col, v);
      }
    }
  }
  if (tws && dtype && T <= 2) {
    __shared__ int last;
    // all 4 waves stored rows of tws: each drains its own stores into L2 before the
    // barrier, so lane 0's agent release (L2 write-back) covers every wave's rows
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the fence's own wait can be dropped
      last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    // the <= 64 block rows of a column loaded at once (clamped rows read, then zeroed), then
    // summed in block order: one memory round trip per column instead of 64
    const int G = (int)gridDim.x;
    for (long k = threadIdx.x; k < (long)T * C; k += 256) {
      const int t = (int)(k / C);
      const long col = k - (long)t * C;
      float r[64];
#pragma unroll
      for (int b = 0; b < 64; ++b) {
        const float x = tws[((long)(b < G ? b : G - 1) * 2 + t) * C + col];
        r[b] = b < G ? x : 0.f;
      }
      float v = 0.f;
#pragma unroll
      for (int b = 0; b < 64; ++b) v += r[b];
      dtype[k] += v;
    }
  }
}

// Word-embedding gradient without float atomics: workgroup g OWNS vocabulary rows
// [16 g, 16 g + 16) and keeps their gradient rows in LDS.  It walks the token ids in
// chunks of 1024 (token order), collects the tokens whose id falls in its range (LDS
// append, then a rank sort by token index inside the chunk), and adds their dh rows in
// token order -- every vocabulary row has exactly one writer and one summation order, so
// the result is bitwise reproducible (the atomic scatter it replaces was neither, and at
// 8192 x 768 took 150 us: 128 workgroups latency-bound on dependent atomics).  Rows that
// received no token are not touched (the arena's zero fill stands).
constexpr int EW_R = 16, EW_CHUNK = 1024, EW_CMAX = 1024;
__global__ void __launch_bounds__(256) embed_word_bwd_kernel(const bf16_t* __restrict__ dh,
                                                             const int32_t* __restrict__ ids,
                                                             float* __restrict__ dword, long M, int C, int V,
                                                             int pad_id) {
  __shared__ float acc[EW_R * EW_CMAX];
  __shared__ int list[EW_CHUNK];
  __shared__ int n_s, touched[EW_R];
  const int tid = threadIdx.x;
  const int v0 = blockIdx.x * EW_R;
  const int C4 = C / 4;
  for (int i = tid; i < EW_R * C; i += 256) acc[i] = 0.f;
  if (tid < EW_R) touched[tid] = 0;
  constexpr int PF = 8;  // chunks whose ids are loaded in one round trip (8192 tokens)
  for (long sbase = 0; sbase < M; sbase += PF * EW_CHUNK) {
   int idr[PF][EW_CHUNK / 256];
#pragma unroll
   for (int c = 0; c < PF; ++c)
#pragma unroll
     for (int u = 0; u < EW_CHUNK / 256; ++u) {
       const long tok = sbase + c * EW_CHUNK + u * 256 + tid;
       idr[c][u] = tok < M ? ids[tok] : -1;
     }
#pragma unroll
   for (int c = 0; c < PF; ++c) {  // unrolled: idr stays in registers
    const long base = sbase + c * EW_CHUNK;
    if (base >= M) break;
    if (tid == 0) n_s = 0;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < EW_CHUNK / 256; ++u) {
      const int id = idr[c][u];
      if (id >= v0 && id < v0 + EW_R && id < V && id != pad_id) {
        const int k = atomicAdd(&n_s, 1);
        list[k] = (u * 256 + tid) | ((id - v0) << 16);
      }
    }
    __syncthreads();
    const int n = n_s;
    if (n == 0) continue;  // uniform: every thread read the same n_s
    // rank sort of this chunk's matches by token index (keys unique)
    int mine[EW_CHUNK / 256], rank[EW_CHUNK / 256];
#pragma unroll
    for (int u = 0; u < EW_CHUNK / 256; ++u) {
      const int i = tid + u * 256;
      mine[u] = i < n ? list[i] : 0;
      rank[u] = 0;
      if (i < n)
        for (int j = 0; j < n; ++j) rank[u] += (list[j] & 0xffff) < (mine[u] & 0xffff);
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < EW_CHUNK / 256; ++u)
      if (tid + u * 256 < n) list[rank[u]] = mine[u];
    __syncthreads();
    // add the dh rows in token order; thread = one 4-column group, 8 rows' loads in flight
    for (int c4 = tid; c4 < C4; c4 += 256) {
      for (int i0 = 0; i0 < n; i0 += 8) {
        float g[8][4];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (i0 + u < n) load4(dh + (base + (list[i0 + u] & 0xffff)) * C + 4 * c4, g[u]);
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (i0 + u < n) {
            float* a = acc + (list[i0 + u] >> 16) * C + 4 * c4;
#pragma unroll
            for (int j = 0; j < 4; ++j) a[j] += g[u][j];
          }
      }
    }
    for (int i = tid; i < n; i += 256) touched[list[i] >> 16] = 1;
    __syncthreads();
   }
  }
  __syncthreads();
  for (int r = 0; r < EW_R; ++r) {
    if (!touched[r]) continue;
    float* o = dword + (long)(v0 + r) * C;
    for (int c4 = tid; c4 < C4; c4 += 256) {
      f4 v = *reinterpret_cast<f4*>(o + 4 * c4);
      v += f4{acc[r * C + 4 * c4], acc[r * C + 4 * c4 + 1], acc[r * C + 4 * c4 + 2], acc[r * C + 4 * c4 + 3]};
      *reinterpret_cast<f4*>(o + 4 * c4) = v;
    }
  }
}

// dpos[s + off] += sum_b dh[b*S + s]  (deterministic, no atomics)
__global__ void __launch_bounds__(256) embed_pos_bwd_kernel(const bf16_t* __restrict__ dh, float* __restrict__ dpos,
                                                            long M, int S, int C, int pos_offset) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;  // over S * C/4
  const int C4 = C / 4;
  if (i >= (long)S * C4) return;
  const int s = (int)(i / C4), c4 = (int)(i - (long)s * C4);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  // 8 batch rows' loads in flight per trip (fixed order: deterministic)
  for (long row0 = s; row0 < M; row0 += 8L * S) {
    float g[8][4];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const long row = row0 + (long)u * S;
      if (row < M) load4(dh + row * C + 4 * c4, g[u]);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (row0 + (long)u * S < M)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] += g[u][j];
  }
  f4* o = reinterpret_cast<f4*>(dpos + (long)(s + pos_offset) * C + 4 * c4);
  f4 v = *o;
  v += f4{acc[0], acc[1], acc[2], acc[3]};
  *o = v;
}

// y = drop(x) (bf16), 8 elements per thread, grid-stride; also used for the backward (same mask).
__global__ void __launch_bounds__(256) dropout_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, long n,
                                                      DropCfg d) {
  const long n8 = n / 8;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    us8 u = *reinterpret_cast<const us8*>(x + 8 * i);
    us8 o;
    float m[8];
    drop_mul4(d, 8 * i, *reinterpret_cast<float(*)[4]>(m));
    drop_mul4(d, 8 * i + 4, *reinterpret_cast<float(*)[4]>(m + 4));
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(u[j]) * m[j]);
    *reinterpret_cast<us8*>(y + 8 * i) = o;
  }
}

__global__ void dropout_mask_kernel(uint8_t* __restrict__ m, long n, long base, DropCfg d) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    m[i] = drop_mul(d, base + i) != 0.f;
}

template <int NV>
int ln_fwd_launch(const bf16_t* x, const bf16_t* res, const float* g, const float* b, bf16_t* y, bf16_t* h, float* mu,
                  float* rs, long M, int C, float eps, DropCfg din, DropCfg dout, const float* xb, hipStream_t s) {
  ln_fwd_kernel<NV><<<ca_cdiv(M, 4), LN_BLK, 0, s>>>(x, res, g, b, y, h, mu, rs, M, C, eps, din, dout, xb);
  return 0;
}

// CLOUD_AMD_LN_BWD16=1 selects the 16-wave form.  Off by default: same kernel time in a
// serialized profile (0.587 vs 0.585 ms per BERT step) but BERT 2.8 % SLOWER with the weight-
// gradient side stream running beside it (7,061 / 7,079 vs 6,879 / 6,881 seq/s with it on,
// profiles/r5_s20/) -- its 1024-thread, 77-KB blocks crowd the side stream's GEMMs off the CUs.
bool ln_bwd16() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CLOUD_AMD_LN_BWD16");
    v = (e && e[0] == '1') ? 1 : 0;
  }
  return v != 0;
}

template <int NV>
int ln_bwd_launch(const bf16_t* dy, const bf16_t* h, const float* mu, const float* rs, const float* g, bf16_t* dh,
                  bf16_t* dx, float* part, int nblk, long M, int C, DropCfg din, DropCfg dout, hipStream_t s) {
  if (ln_bwd16() && C <= 1344) {
    ln_bwd16_kernel<NV><<<nblk, 1024, 25 * C * sizeof(float), s>>>(dy, h, mu, rs, g, dh, dx, part, M, C, din, dout);
    return 0;
  }
  ln_bwd_kernel<NV><<<nblk, LN_BLK, 12 * C * sizeof(float), s>>>(dy, h, mu, rs, g, dh, dx, part, M, C, din, dout);
  return 0;
}

// LayerNorm-backward blocks (4 rows each per trip; each block leaves one [3][C] partial row
// for col_finalize).  Measured at M = 8192, C = 768: 512 blocks 19-23 us, 1024 blocks 25-26 us.
// (An 8-wave block taking two rows per wave per trip -- 4,096 waves instead of 2,048 -- made
// BERT 1.5 % SLOWER: 6,774 / 6,790 vs 6,866 / 6,899 seq/s, profiles/r5_s4/.)
int ln_nblk(long M) {
  long b = (M + 3) / 4;
  return (int)(b < 512 ? b : 512);
}

// Keras Dense / Conv2D backward through a fused activation (ops/dense.py): g = dy * act'(.)
// in one pass, bf16 in / bf16 out, with the zero column padding of dy to the layer's padded
// width folded in (the 10-way softmax head runs its GEMMs 16 wide).  relu / elu / tanh take
// act' from the saved OUTPUT y; gelu from the saved pre-activation (erf form, as the
// forward epilogue).  src and out are [M][Np]; dy is [M][ld_dy] with N <= Np real columns.
__global__ void __launch_bounds__(256) act_grad_kernel(const bf16_t* __restrict__ dy, long ld_dy, int N,
                                                       const bf16_t* __restrict__ src, bf16_t* __restrict__ out,
                                                       long M, int Np, int act) {
  const int cpr = Np / 8;
  const long total = M * cpr;
  const bool fast = (N == Np) && (ld_dy % 8 == 0);
  for (long c = (long)blockIdx.x * blockDim.x + threadIdx.x; c < total; c += (long)gridDim.x * blockDim.x) {
    const long m = c / cpr;
    const int n0 = (int)(c - m * cpr) * 8;
    float g[8];
    if (fast) {
      const us8 d = *reinterpret_cast<const us8*>(dy + m * ld_dy + n0);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = bf2f(d[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = (n0 + j < N) ? bf2f(dy[m * ld_dy + n0 + j]) : 0.f;
    }
    const us8 sv = *reinterpret_cast<const us8*>(src + m * Np + n0);
    us8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = bf2f(sv[j]);
      float d;
      switch (act) {
        case ca::ACT_RELU: d = v > 0.f ? 1.f : 0.f; break;
        case ca::ACT_ELU: d = v > 0.f ? 1.f : v + 1.f; break;
        case ca::ACT_TANH: d = 1.f - v * v; break;
        case ca::ACT_GELU: d = ca::act_grad(ca::ACT_GELU, v); break;
        default: d = 1.f;
      }
      o[j] = f2bf(g[j] * d);
    }
    *reinterpret_cast<us8*>(out + m * Np + n0) = o;
  }
}

// Zero-pad the columns of a row-major matrix to a multiple the MFMA tiles take (Keras
// layers with Cin = 1 / 3 or a 10-way head): out[r][c] = c < cols ? in[r * ld + c] : 0,
// out row stride cols_out; 2- or 4-byte elements.  One launch instead of F.pad's fill + copy.
struct PadJob {
  const void* in;
  void* out;
  long ld, rows, rows_out;
  int cols, cols_out, eb;
};
struct PadJobs {
  PadJob j[4];
};

// several pad_cols jobs in one launch (blockIdx.y = job): a layer's padded input, weight
// and bias cost one dispatch
__global__ void __launch_bounds__(256) pad_cols_multi_kernel(PadJobs jobs) {
  const PadJob& J = jobs.j[blockIdx.y];
  const long n = J.rows_out * J.cols_out;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const long r = i / J.cols_out;
    const int c = (int)(i - r * J.cols_out);
    const bool ok = c < J.cols && r < J.rows;
    if (J.eb == 2)
      reinterpret_cast<uint16_t*>(J.out)[i] = ok ? reinterpret_cast<const uint16_t*>(J.in)[r * J.ld + c] : 0;
    else
      reinterpret_cast<uint32_t*>(J.out)[i] = ok ? reinterpret_cast<const uint32_t*>(J.in)[r * J.ld + c] : 0u;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) pad_cols_kernel(const T* __restrict__ in, long ld, int cols,
                                                       T* __restrict__ out, int cols_out, long rows, long rows_out) {
  const long n = rows_out * cols_out;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const long r = i / cols_out;
    const int c = (int)(i - r * cols_out);
    out[i] = (c < cols && r < rows) ? in[r * ld + c] : (T)0;
  }
}

// Accumulate the [rows][cols] top-left block of an fp32 [rows_in][ld_in] gradient into a
// parameter-shaped arena slot (bf16 or fp32): the padded Keras layers (Cin 1 / 3, 10-way
// heads) compute their weight gradients on the padded shape -- one launch instead of a
// slice copy, a cast and an add.
template <typename T>
__global__ void __launch_bounds__(256) slice_acc_kernel(const float* __restrict__ in, long ld_in,
                                                        T* __restrict__ out, long rows, int cols) {
  const long n = rows * cols;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const long r = i / cols;
    const int c = (int)(i - r * cols);
    if constexpr (sizeof(T) == 2) {
      out[i] = f2bf(bf2f(out[i]) + in[r * ld_in + c]);
    } else {
      out[i] += in[r * ld_in + c];
    }
  }
}

}  // namespace

extern "C" {

long ca_ln_workspace_floats(long M, int C) { return (long)ln_nblk(M) * 3 * C; }

// y = drop_out(LN(res + drop_in(x + xbias))); h_out (optional) keeps the pre-norm sum for the
// backward; xbias (optional, fp32 [C]) is the bias of the GEMM that produced x.
int ca_ln_fwd(const bf16_t* x, const bf16_t* res, const float* gamma, const float* beta, bf16_t* y, bf16_t* h_out,
              float* mean, float* rstd, long M, int C, float eps, float p_in, uint64_t seed_in, float p_out,
              uint64_t seed_out, const float* xbias, hipStream_t s) {
  if (C % 4 != 0 || C > 2048) return -1;
  const DropCfg din = make_drop(p_in, seed_in), dout = make_drop(p_out, seed_out);
  const int nv = (C / 4 + 63) / 64;
  int rc;
  switch (nv) {
    case 1: rc = ln_fwd_launch<1>(x, res, gamma, beta, y, h_out, mean, rstd, M, C, eps, din, dout, xbias, s); break;
    case 2: rc = ln_fwd_launch<2>(x, res, gamma, beta, y, h_out, mean, rstd, M, C, eps, din, dout, xbias, s); break;
    case 3: rc = ln_fwd_launch<3>(x, res, gamma, beta, y, h_out, mean, rstd, M, C, eps, din, dout, xbias, s); break;
    case 4: rc = ln_fwd_launch<4>(x, res, gamma, beta, y, h_out, mean, rstd, M, C, eps, din, dout, xbias, s); break;
    default: rc = ln_fwd_launch<8>(x, res, gamma, beta, y, h_out, mean, rstd, M, C, eps, din, dout, xbias, s); break;
  }
  if (rc) return rc;
  CA_LAUNCH_CHECK();
  return 0;
}

// dh = LN'(drop_out'(dy)); dx = drop_in'(dh) when dx != null; dgamma/dbeta (+)= column sums;
// dsum (optional) (+)= column sums of dx (or dh): the upstream dense layer's bias gradient.
int ca_ln_bwd(const bf16_t* dy, const bf16_t* h, const float* mean, const float* rstd, const float* gamma, bf16_t* dh,
              bf16_t* dx, float* dgamma, float* dbeta, int accumulate, float* ws, long M, int C, float p_in,
              uint64_t seed_in, float p_out, uint64_t seed_out, hipStream_t s, float* dsum) {
  if (C % 4 != 0 || C > 1344) return -1;  // 12*C floats of dynamic LDS stay within 64 KB
  const DropCfg din = make_drop(p_in, seed_in), dout = make_drop(p_out, seed_out);
  const int nv = (C / 4 + 63) / 64;
  const int nblk = ln_nblk(M);
  switch (nv) {
    case 1: ln_bwd_launch<1>(dy, h, mean, rstd, gamma, dh, dx, ws, nblk, M, C, din, dout, s); break;
    case 2: ln_bwd_launch<2>(dy, h, mean, rstd, gamma, dh, dx, ws, nblk, M, C, din, dout, s); break;
    case 3: ln_bwd_launch<3>(dy, h, mean, rstd, gamma, dh, dx, ws, nblk, M, C, din, dout, s); break;
    case 4: ln_bwd_launch<4>(dy, h, mean, rstd, gamma, dh, dx, ws, nblk, M, C, din, dout, s); break;
    default: ln_bwd_launch<8>(dy, h, mean, rstd, gamma, dh, dx, ws, nblk, M, C, din, dout, s); break;
  }
  CA_LAUNCH_CHECK();
  // accumulate < 0: the caller finalises the [nblk][3][C] partials in ws itself (batched
  // finalisation, gradfin.hip)
  if (accumulate >= 0 && (dgamma || dbeta || dsum)) {
    col_finalize_kernel<<<ca_cdiv((dsum ? 3 : 2) * C, 16), 256, 0, s>>>(ws, nblk, 3L * C, C, dgamma, dbeta,
                                                                        accumulate, dsum);
    CA_LAUNCH_CHECK();
  }
  return 0;
}

long ca_colsum_workspace_floats(long M, int N) { return 256L * N; }

// out[n] (+)= sum_m x[m*ld + n]  (bias gradient), N % 8 == 0; ws >= 64*N floats.
int ca_pad_cols(const void* in, long ld, int cols, void* out, int cols_out, long rows, long rows_out, int elem_bytes,
                hipStream_t s) {
  if (cols > cols_out || rows <= 0 || rows > rows_out) return -1;
  const int g = ca_stream_grid(rows_out * cols_out, 256);
  if (elem_bytes == 2)
    pad_cols_kernel<uint16_t><<<g, 256, 0, s>>>((const uint16_t*)in, ld, cols, (uint16_t*)out, cols_out, rows,
                                                 rows_out);
  else if (elem_bytes == 4)
    pad_cols_kernel<uint32_t><<<g, 256, 0, s>>>((const uint32_t*)in, ld, cols, (uint32_t*)out, cols_out, rows,
                                                 rows_out);
  else
    return -1;
  CA_LAUNCH_CHECK();
  return 0;
}

// jobs: n x [in, ld, cols, out, cols_out, rows, rows_out, elem_bytes] (n <= 4)
int ca_pad_cols_multi(const long* jobs, int n, hipStream_t s) {
  if (n < 1 || n > 4) return -1;
  PadJobs P{};
  long most = 1;
  for (int k = 0; k < n; ++k) {
    const long* q = jobs + 8 * k;
    PadJob& J = P.j[k];
    J.in = reinterpret_cast<const void*>(q[0]);
    J.ld = q[1];
    J.cols = (int)q[2];
    J.out = reinterpret_cast<void*>(q[3]);
    J.cols_out = (int)q[4];
    J.rows = q[5];
    J.rows_out = q[6];
    J.eb = (int)q[7];
    if (J.cols > J.cols_out || J.rows > J.rows_out || (J.eb != 2 && J.eb != 4)) return -1;
    if (J.rows_out * J.cols_out > most) most = J.rows_out * J.cols_out;
  }
  pad_cols_multi_kernel<<<dim3(ca_stream_grid(most, 256), n), 256, 0, s>>>(P);
  CA_LAUNCH_CHECK();
  return 0;
}

int ca_slice_acc(const float* in, long ld_in, void* out, int out_bf16, long rows, int cols, hipStream_t s) {
  if (rows <= 0 || cols <= 0 || ld_in < cols) return -1;
  const int g = ca_stream_grid(rows * cols, 256);
  if (out_bf16) slice_acc_kernel<bf16_t><<<g, 256, 0, s>>>(in, ld_in, (bf16_t*)out, rows, cols);
  else slice_acc_kernel<float><<<g, 256, 0, s>>>(in, ld_in, (float*)out, rows, cols);
  CA_LAUNCH_CHECK();
  return 0;
}

int ca_act_grad(const bf16_t* dy, long ld_dy, int N, const bf16_t* src, bf16_t* out, long M, int Np, int act,
                hipStream_t s) {
  if (Np % 8 != 0 || N > Np || M <= 0) return -1;
  act_grad_kernel<<<ca_stream_grid(M * (Np / 8), 256), 256, 0, s>>>(dy, ld_dy, N, src, out, M, Np, act);
  CA_LAUNCH_CHECK();
  return 0;
}

int ca_colsum(const bf16_t* x, long M, int N, long ld, float* out, int accumulate, float* ws, hipStream_t s) {
  if (N % 8 != 0) return -1;
  int ry = (int)((M + 63) / 64);
  if (ry > 256) ry = 256;
  if (ry < 1) ry = 1;
  dim3 grid(ca_cdiv(N, 256), ry);
  if (ry == 1 && accumulate >= 0) {  // <= 64 rows (a Keras Dense bias): one launch, no finalize
    colsum_part_kernel<<<grid, 256, 0, s>>>(x, M, N, ld, ws, out, accumulate);
    CA_LAUNCH_CHECK();
    return 0;
  }
  colsum_part_kernel<<<grid, 256, 0, s>>>(x, M, N, ld, ws);
  CA_LAUNCH_CHECK();
  if (accumulate < 0) return 0;  // partials [ry][N] left in ws for a batched finalisation
  col_finalize_kernel<<<ca_cdiv(N, 16), 256, 0, s>>>(ws, ry, N, N, out, nullptr, accumulate);
  CA_LAUNCH_CHECK();
  return 0;
}

int ca_embed_sum(const int32_t* ids, const int32_t* tts, const float* word, const float* pos, const float* type,
                 bf16_t* h, long M, int S, int C, int pos_offset, hipStream_t s) {
  if (C % 4 != 0) return -1;
  embed_sum_kernel<<<ca_cdiv(M, 4), 256, 0, s>>>(ids, tts, word, pos, type, h, M, S, C, pos_offset);
  CA_LAUNCH_CHECK();
  return 0;
}

// tws / tk: the deterministic token-type reduction's workspace ([64 blocks][2][C] fp32) and
// its ticket (zero at launch; the kernel's last block resets it), owned by the caller --
// one per stream, from the caching allocator (cloud_amd/ops/raw.py embed_bwd).
// Returns 0, or 1 when a gradient took the order-dependent float-atomic path (more than
// two token types, rows wider than the owner kernel holds, or no workspace given).
int ca_embed_bwd(const bf16_t* dh, const int32_t* ids, const int32_t* tts, float* dword, float* dpos, float* dtype,
                 long M, int S, int C, int T, int pos_offset, int pad_id, int V, float* tws, unsigned* tk,
                 hipStream_t s) {
  if (C % 4 != 0) return -1;
  int nondet = 0;
  // word rows: the owner kernel (deterministic) when its LDS rows hold C; token types (and
  // wide rows) on the segment-pre-reduced atomic scatter
  const bool owner = dword && C <= EW_CMAX && V > 0 && M < (1L << 31);
  if (owner) {
    embed_word_bwd_kernel<<<ca_cdiv(V, EW_R), 256, 0, s>>>(dh, ids, dword, M, C, V, pad_id);
    CA_LAUNCH_CHECK();
  }
  if ((dword && !owner) || dtype) {
    // each wave takes EB_RW consecutive rows per trip; type-only: at most 64 blocks (fewer
    // atomics per column, see the kernel)
    int grid = ca_cdiv(M, 4 * EB_RW);
    if (!(dword && !owner) && grid > 64) grid = 64;
    if (grid < 1) grid = 1;
    const bool det_type = dtype && T <= 2 && !(dword && !owner) && tws && tk;
    if ((dword && !owner) || (dtype && !det_type)) nondet = 1;
    embed_bwd_kernel<<<grid, 256, 0, s>>>(dh, ids, tts, owner ? nullptr : dword, dtype, M, C, T, pad_id,
                                          det_type ? tws : nullptr, det_type ? tk : nullptr);
    CA_LAUNCH_CHECK();
  }
  if (dpos) {
    embed_pos_bwd_kernel<<<ca_cdiv((long)S * (C / 4), 256), 256, 0, s>>>(dh, dpos, M, S, C, pos_offset);
    CA_LAUNCH_CHECK();
  }
  return nondet;
}

int ca_dropout(const bf16_t* x, bf16_t* y, long n, float p, uint64_t seed, hipStream_t s) {
  if (n % 8 != 0) return -1;
  dropout_kernel<<<ca_stream_grid(n / 8, 256), 256, 0, s>>>(x, y, n, make_drop(p, seed));
  CA_LAUNCH_CHECK();
  return 0;
}

int ca_dropout_mask(uint8_t* m, long n, long base, float p, uint64_t seed, hipStream_t s) {
  dropout_mask_kernel<<<ca_stream_grid(n, 256), 256, 0, s>>>(m, n, base, make_drop(p, seed));
  CA_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
