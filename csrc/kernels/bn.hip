// Training-mode BatchNorm (+ residual add + ReLU) for NHWC bf16 activations
// viewed as a row-major [M = N*H*W, C] matrix (K10 in SURVEY.md section 2.7).
//
// Forward  : stats (1 read)  -> finalize (per-channel, tiny) -> apply (1 read + 1 write
//            [+1 read residual]).
// Backward : reduce (dy, x + ReLU bitmask) -> finalize -> apply (same reads, 1-2
//            writes); the ReLU mask is the 1-bit-per-channel map written by the
//            forward apply (or recomputed from y when none was kept); the residual
//            gradient is emitted by the same pass.
//
// Tiling: a block is 256 threads = TW column-vectors (8 channels, 16 B each) x RP
// rows; each thread owns ONE column vector for the whole launch (so per-channel
// coefficients live in registers) and walks rows with stride RP.  Partial sums
// go to a [nchunks][C] fp32 workspace (deterministic, no atomics) and are
// combined in double precision by the finalize kernel.
#include "ca_common.h"

#include <mutex>

namespace {

constexpr int BLK = 256;

struct Tiling {
  int CT, TW, RP, ncol, nchunks;
  long rows_per_chunk;
  int ilv;  // apply passes: row groups of RP rows dealt round-robin to the blocks (grid stride)
};

// total: workgroups wanted over all column blocks; cap: row chunks at most.  The
// reduction kernels keep (2048, 1024): their partials are [nchunks][C].
__host__ __device__ inline Tiling make_tiling(long M, int C, int total = 2048, int cap = 1024) {
  Tiling t;
  t.CT = C / 8;
  t.TW = t.CT < 64 ? t.CT : 64;
  t.RP = BLK / t.TW;
  t.ncol = (t.CT + t.TW - 1) / t.TW;
  long maxchunks = (M + t.RP - 1) / t.RP;
  long want = total / t.ncol;
  if (want < 1) want = 1;
  if (want > maxchunks) want = maxchunks;
  if (want > cap) want = cap;
  t.nchunks = (int)want;
  long rpc = (M + t.nchunks - 1) / t.nchunks;
  rpc = ((rpc + t.RP - 1) / t.RP) * t.RP;
  t.rows_per_chunk = rpc;
  t.ilv = 0;
  t.nchunks = (int)((M + rpc - 1) / rpc);
  return t;
}

// Elementwise apply passes need no partials, so their grid is sized for the HBM stream
// alone: CLOUD_AMD_BN_APPLY_BLOCKS workgroups in total (0 = the reduction tiling);
// RP-row groups are dealt round-robin (one contiguous sweep by the blocks in flight:
// bwd apply 4.8-5.1 -> 5.5-5.6 TB/s on the ResNet-50 shapes, bench/bn_apply_bw.py);
// CLOUD_AMD_BN_APPLY_ILV=0 keeps one contiguous row chunk per block (A/B runs).
inline Tiling apply_tiling(long M, int C) {
  static int blocks = -1, ilv = 1;
  if (blocks < 0) {
    const char* e = getenv("CLOUD_AMD_BN_APPLY_BLOCKS");
    blocks = e ? atoi(e) : 0;
    if (blocks < 0) blocks = 0;
    const char* f = getenv("CLOUD_AMD_BN_APPLY_ILV");
    ilv = (f && f[0] == '0') ? 0 : 1;
  }
  Tiling t = blocks ? make_tiling(M, C, blocks, blocks) : make_tiling(M, C);
  t.ilv = ilv;
  return t;
}

__device__ __forceinline__ void ld8bf(const bf16_t* p, float (&o)[8]) {
  us8 v = *reinterpret_cast<const us8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = bf2f(v[j]);
}
__device__ __forceinline__ void st8bf(bf16_t* p, const float (&o)[8]) {
  us8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = f2bf(o[j]);
  *reinterpret_cast<us8*>(p) = v;
}

// Reduce two per-thread 8-vectors over the RP threads sharing a column, write
// the block's partial to ws[chunk][C] (a) and ws[nchunks + chunk][C] (b).
__device__ __forceinline__ void block_col_reduce(float (&a)[8], float (&b)[8], const Tiling& t,
                                                 int tx, int ty, int vc, int chunk, int C,
                                                 float* __restrict__ ws) {
  __shared__ float sa[BLK * 8];
  __shared__ float sb[BLK * 8];
  const int tid = threadIdx.x;
#pragma unroll
  for (int j = 0; j < 8; ++j) { sa[j * BLK + tid] = a[j]; sb[j * BLK + tid] = b[j]; }
  __syncthreads();
  // threads (tx, ty) sum channels j = ty, ty+RP, ... of column tx over the RP rows
  if (vc < t.CT) {
    for (int j = ty; j < 8; j += t.RP) {
      float ra = 0.f, rb = 0.f;
      for (int r = 0; r < t.RP; ++r) {
        ra += sa[j * BLK + r * t.TW + tx];
        rb += sb[j * BLK + r * t.TW + tx];
      }
      const int c = vc * 8 + j;
      ws[(long)chunk * C + c] = ra;
      ws[(long)(t.nchunks + chunk) * C + c] = rb;
    }
  }
}

// Sum the [nchunks][C] partials of channel c with one WAVE (lanes stride over
// chunks, fp64 accumulation, shuffle reduction).  Returns the totals in every lane.
__device__ __forceinline__ void wave_chunk_sum(const float* __restrict__ ws, int nchunks, long stride_k, long off_q,
                                               int c, double& a, double& b) {
  const int lane = threadIdx.x & 63;
  double sa = 0.0, sb = 0.0;
#pragma unroll 8
  for (int k = lane; k < nchunks; k += 64) {
    sa += ws[(long)k * stride_k + c];
    sb += ws[(long)k * stride_k + off_q + c];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    sa += __shfl_xor(sa, o, 64);
    sb += __shfl_xor(sb, o, 64);
  }
  a = sa;
  b = sb;
}

// First level of the statistics reduction when there are many partial rows
// (e.g. one per 128-row GEMM tile: 6272 for a 56x56x256 batch-256 layer):
// block = 64 channels x 4 part-lanes, blockIdx.y = group g; out[g][0|1][C]
// holds the group's sums of the two quantities (deterministic order).  The
// finalize kernels then reduce only G rows -- enough blocks in flight instead
// of one latency-bound wave per channel walking thousands of rows.
__global__ void __launch_bounds__(256) chunk_group_reduce_kernel(const float* __restrict__ ws, int nchunks,
                                                                 long stride_k, long off_q, int C,
                                                                 float* __restrict__ out) {
  __shared__ float ra[4][64], rb[4][64];
  const int cl = threadIdx.x & 63, pl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int G = gridDim.y, g = blockIdx.y;
  float a = 0.f, b = 0.f;
  if (c < C) {
#pragma unroll 4
    for (int k = g * 4 + pl; k < nchunks; k += G * 4) {
      a += ws[(long)k * stride_k + c];
      b += ws[(long)k * stride_k + off_q + c];
    }
  }
  ra[pl][cl] = a;
  rb[pl][cl] = b;
  __syncthreads();
  if (pl != 0 || c >= C) return;
  out[(long)g * 2 * C + c] = (ra[0][cl] + ra[1][cl]) + (ra[2][cl] + ra[3][cl]);
  out[(long)g * 2 * C + C + c] = (rb[0][cl] + rb[1][cl]) + (rb[2][cl] + rb[3][cl]);
}

// ~64 partial rows per group, at most 512 groups (the [512][2][C] group workspace the
// callers pass).  A 56x56 layer at batch 1024 has 25,088 tile rows: 64 groups left 64
// workgroups walking 392 rows each (18-22 us, latency-bound); 392 groups take ~5 us.
int group_count(int nchunks) {
  static int cap = -1;
  if (cap < 0) {  // CLOUD_AMD_BN_GROUPS_MAX (A/B runs; 64 = the earlier fixed cap)
    const char* e = getenv("CLOUD_AMD_BN_GROUPS_MAX");
    cap = e ? atoi(e) : 512;
    if (cap < 1 || cap > 512) cap = 512;
  }
  int g = (nchunks + 63) / 64;
  return g < 1 ? 1 : (g > cap ? cap : g);
}

__global__ void __launch_bounds__(BLK) bn_stats_kernel(const bf16_t* __restrict__ x, long M, int C,
                                                      float* __restrict__ ws) {
  const Tiling t = make_tiling(M, C);
  const int tx = threadIdx.x % t.TW, ty = threadIdx.x / t.TW;
  const int vc = blockIdx.x * t.TW + tx;
  const int chunk = blockIdx.y;
  float s[8] = {0}, q[8] = {0};
  if (vc < t.CT) {
    const long r0 = (long)chunk * t.rows_per_chunk;
    long r1 = r0 + t.rows_per_chunk;
    if (r1 > M) r1 = M;
    const bf16_t* base = x + (long)vc * 8;
    long r = r0 + ty;
    for (; r + 3 * t.RP < r1; r += 4 * t.RP) {
      float v0[8], v1[8], v2[8], v3[8];
      ld8bf(base + r * C, v0);
      ld8bf(base + (r + t.RP) * C, v1);
      ld8bf(base + (r + 2 * t.RP) * C, v2);
      ld8bf(base + (r + 3 * t.RP) * C, v3);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[j] += (v0[j] + v1[j]) + (v2[j] + v3[j]);
        q[j] += (v0[j] * v0[j] + v1[j] * v1[j]) + (v2[j] * v2[j] + v3[j] * v3[j]);
      }
    }
    for (; r < r1; r += t.RP) {
      float v0[8];
      ld8bf(base + r * C, v0);
#pragma unroll
      for (int j = 0; j < 8; ++j) { s[j] += v0[j]; q[j] += v0[j] * v0[j]; }
    }
  }
  block_col_reduce(s, q, t, tx, ty, vc, chunk, C, ws);
}

// Per-channel finalize of the forward statistics.
//   save_mean/save_rstd : fp32 [C] (needed by backward)
//   scale/shift         : fp32 [C], y = x*scale + shift
//   running stats updated in place when non-null (unbiased variance).
struct FwdFin {
  long M;
  const float *gamma, *beta;
  float eps, momentum;
  float *run_mean, *run_var, *save_mean, *save_rstd, *scale, *shift;
  __device__ void operator()(int c, double s, double q) const {
    const double mean = s / (double)M;
    double var = q / (double)M - mean * mean;
    if (var < 0.0) var = 0.0;
    const float rstd = (float)(1.0 / sqrt(var + (double)eps));
    const float g = gamma ? gamma[c] : 1.f;
    const float b = beta ? beta[c] : 0.f;
    save_mean[c] = (float)mean;
    save_rstd[c] = rstd;
    scale[c] = g * rstd;
    shift[c] = b - (float)mean * g * rstd;
    if (run_mean) {
      const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
      run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (float)mean;
      run_var[c] = (1.f - momentum) * run_var[c] + momentum * (float)unb;
    }
  }
};

__global__ void bn_fwd_finalize_kernel(const float* __restrict__ ws, int nchunks, long stride_k, long off_q,
                                       int C, const FwdFin F) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= C) return;
  double s, q;
  wave_chunk_sum(ws, nchunks, stride_k, off_q, c, s, q);
  if ((threadIdx.x & 63) != 0) return;
  F(c, s, q);
}

// y = act(x*scale + shift [+ res]); with a ReLU, optionally also the ReLU
// bitmask (1 byte per 8 channels: bit j = y[c0+j] > 0) so the backward reads
// 1/16 of the bytes of y for its mask.
template <bool RELU, bool RES>
__global__ void __launch_bounds__(BLK) bn_apply_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                      const float* __restrict__ scale, const float* __restrict__ shift,
                                                      bf16_t* __restrict__ y, uint8_t* __restrict__ mask, long M,
                                                      int C, const Tiling tl) {
  const Tiling& t = tl;
  const int tx = threadIdx.x % t.TW, ty = threadIdx.x / t.TW;
  const int vc = blockIdx.x * t.TW + tx;
  if (vc >= t.CT) return;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sc[j] = scale[vc * 8 + j]; sh[j] = shift[vc * 8 + j]; }
  // contiguous row chunk per block, or (ilv) RP-row groups dealt round-robin so that the
  // blocks in flight sweep one contiguous span instead of ~nchunks far-apart streams
  const long step = t.ilv ? (long)gridDim.y * t.RP : t.RP;
  const long r0 = t.ilv ? (long)blockIdx.y * t.RP : (long)blockIdx.y * t.rows_per_chunk;
  long r1 = t.ilv ? M : r0 + t.rows_per_chunk;
  if (r1 > M) r1 = M;
  const long off0 = (long)vc * 8;
  for (long r = r0 + ty; r < r1; r += step) {
    const long o = r * C + off0;
    float v[8];
    ld8bf(x + o, v);
    float rv[8];
    if (RES) ld8bf(res + o, rv);
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float z = bn_affine(v[j], sc[j], sh[j]);
      if (RES) z += rv[j];
      if (RELU) {
        z = fmaxf(z, 0.f);
        bits |= (z > 0.f ? 1u : 0u) << j;
      }
      v[j] = z;
    }
    st8bf(y + o, v);
    if (RELU && mask) mask[r * t.CT + vc] = (uint8_t)bits;
  }
}

// y = act(x*scale + shift + (r*rscale + rshift)): the residual is the INPUT of another
// BatchNorm (a projection shortcut) whose affine is applied on the fly, so that BN's own
// output is never written or read back.
template <bool RELU>
__global__ void __launch_bounds__(BLK) bn_apply_resbn_kernel(const bf16_t* __restrict__ x,
                                                            const bf16_t* __restrict__ r,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift,
                                                            const float* __restrict__ rscale,
                                                            const float* __restrict__ rshift, bf16_t* __restrict__ y,
                                                            uint8_t* __restrict__ mask, long M, int C, const Tiling tl) {
  const Tiling& t = tl;
  const int tx = threadIdx.x % t.TW, ty = threadIdx.x / t.TW;
  const int vc = blockIdx.x * t.TW + tx;
  if (vc >= t.CT) return;
  float sc[8], sh[8], rs[8], rh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = scale[vc * 8 + j];
    sh[j] = shift[vc * 8 + j];
    rs[j] = rscale[vc * 8 + j];
    rh[j] = rshift[vc * 8 + j];
  }
  const long step = t.ilv ? (long)gridDim.y * t.RP : t.RP;
  const long r0 = t.ilv ? (long)blockIdx.y * t.RP : (long)blockIdx.y * t.rows_per_chunk;
  long r1 = t.ilv ? M : r0 + t.rows_per_chunk;
  if (r1 > M) r1 = M;
  const long off0 = (long)vc * 8;
  for (long rr = r0 + ty; rr < r1; rr += step) {
    const long o = rr * C + off0;
    float v[8], rv[8];
    ld8bf(x + o, v);
    ld8bf(r + o, rv);
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      // the shortcut BN output rounded to bf16 exactly as if it had been stored, so the
      // block stays bit-compatible with the op-by-op path
      const float idn = bf2f(f2bf(bn_affine(rv[j], rs[j], rh[j])));
      float z = bn_affine(v[j], sc[j], sh[j]) + idn;
      if (RELU) {
        z = fmaxf(z, 0.f);
        bits |= (z > 0.f ? 1u : 0u) << j;
      }
      v[j] = z;
    }
    st8bf(y + o, v);
    if (RELU && mask) mask[rr * t.CT + vc] = (uint8_t)bits;
  }
}

__device__ __forceinline__ void relu_gate(float (&d)[8], const bf16_t* __restrict__ y, const uint8_t* __restrict__ mask,
                                          long r, long o, int CT, int vc) {
  if (mask) {
    const uint32_t m = mask[r * CT + vc];
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = ((m >> j) & 1u) ? d[j] : 0.f;
  } else {
    float yv[8];
    ld8bf(y + o, yv);
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = yv[j] > 0.f ? d[j] : 0.f;
  }
}

// Backward reduce: dz = dy * relu'(y) (from the bitmask, or y when no mask);
// partial sums of dz and dz*xhat.
template <bool RELU>
__global__ void __launch_bounds__(BLK) bn_bwd_reduce_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y,
                                                           const uint8_t* __restrict__ mask,
                                                           const bf16_t* __restrict__ x,
                                                           const float* __restrict__ mean, const float* __restrict__ rstd,
                                                           long M, int C, float* __restrict__ ws) {
  const Tiling t = make_tiling(M, C);
  const int tx = threadIdx.x % t.TW, ty = threadIdx.x / t.TW;
  const int vc = blockIdx.x * t.TW + tx;
  const int chunk = blockIdx.y;
  float sd[8] = {0}, sdx[8] = {0};
  if (vc < t.CT) {
    float mu[8], rs[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { mu[j] = mean[vc * 8 + j]; rs[j] = rstd[vc * 8 + j]; }
    const long r0 = (long)chunk * t.rows_per_chunk;
    long r1 = r0 + t.rows_per_chunk;
    if (r1 > M) r1 = M;
    const long off0 = (long)vc * 8;
    long r = r0 + ty;
    for (; r + t.RP < r1; r += 2 * t.RP) {
      const long o0 = r * C + off0, o1 = (r + t.RP) * C + off0;
      float d0[8], x0[8], d1[8], x1[8];
      ld8bf(dy + o0, d0);
      ld8bf(x + o0, x0);
      ld8bf(dy + o1, d1);
      ld8bf(x + o1, x1);
      if (RELU) {
        relu_gate(d0, y, mask, r, o0, t.CT, vc);
        relu_gate(d1, y, mask, r + t.RP, o1, t.CT, vc);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sd[j] += d0[j] + d1[j];
        sdx[j] += d0[j] * (x0[j] - mu[j]) * rs[j] + d1[j] * (x1[j] - mu[j]) * rs[j];
      }
    }
    for (; r < r1; r += t.RP) {
      const long o0 = r * C + off0;
      float d0[8], x0[8];
      ld8bf(dy + o0, d0);
      ld8bf(x + o0, x0);
      if (RELU) relu_gate(d0, y, mask, r, o0, t.CT, vc);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sd[j] += d0[j];
        sdx[j] += d0[j] * (x0[j] - mu[j]) * rs[j];
      }
    }
  }
  block_col_reduce(sd, sdx, t, tx, ty, vc, chunk, C, ws);
}

// dgamma = sum(dz*xhat), dbeta = sum(dz); coefficients so that
// dx = A*dz + B*x + D.
struct BwdFin {
  long M;
  int C;
  const float *gamma, *mean, *rstd;
  float *dgamma, *dbeta, *coef;
  int accum, raw_moments;
  __device__ void operator()(int c, double sd, double sdx) const {
    // partials from a GEMM epilogue hold sum(dz*x): sum(dz*xhat) = rstd*(sum(dz*x) - mean*sum(dz))
    if (raw_moments) sdx = (double)rstd[c] * (sdx - (double)mean[c] * sd);
    // accum: parameter grads are summed into (flat arena slots), not overwritten
    if (dgamma) dgamma[c] = (float)sdx + (accum ? dgamma[c] : 0.f);
    if (dbeta) dbeta[c] = (float)sd + (accum ? dbeta[c] : 0.f);
    const double g = gamma ? gamma[c] : 1.0;
    const double rs = rstd[c], mu = mean[c];
    const double k1 = g * rs;
    const double a = sd / (double)M, b = sdx / (double)M;
    coef[c] = (float)k1;                                    // A
    coef[C + c] = (float)(-k1 * b * rs);                    // B
    coef[2 * C + c] = (float)(-k1 * a + k1 * b * rs * mu);  // D
  }
};

// Group reduction AND finalize in one launch (one dispatch per BatchNorm instead of two):
// block = 64 channels x 16 part-lanes (1024 threads); block (x, g) sums partial rows
// [g * FIN_RPG, (g + 1) * FIN_RPG) of its 64 channels into group row g, then counts itself on a
// per-column-block ticket (agent-scope release); the block that arrives last for its 64 channels
// (acquire) sums the G group rows in a FIXED order -- the same result whichever block finishes
// last -- runs the finalize and re-arms the ticket.  No block ever waits for another.  Groups
// are 512 rows by default so the last block's pass is a single round of loads (G <= 49 at
// 25,088 rows).
constexpr int FIN_PL = 16;

// partial rows per group (CLOUD_AMD_BN_FIN_RPG, 64..512, default 512): fewer rows per group =
// more blocks reading the partials at once, and more group rows for the last block to sum
int fin_rpg() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CLOUD_AMD_BN_FIN_RPG");
    const int r = e ? atoi(e) : 512;
    v = (r >= 64 && r <= 512 && r % FIN_PL == 0) ? r : 512;
  }
  return v;
}

template <class FIN>
__global__ void __launch_bounds__(64 * FIN_PL) group_finalize_kernel(const float* __restrict__ ws, int nchunks,
                                                                     long stride_k, long off_q, int C, int rpg,
                                                                     float* __restrict__ gws,
                                                                     unsigned* __restrict__ tickets, const FIN F) {
  __shared__ float ra[FIN_PL][64], rb[FIN_PL][64];
  __shared__ double da[FIN_PL][64], db[FIN_PL][64];
  __shared__ int last;
  const int tid = threadIdx.x, cl = tid & 63, pl = tid >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int G = gridDim.y, g = blockIdx.y;
  float a = 0.f, b = 0.f;
  if (c < C) {
    int k1 = (g + 1) * rpg;
    if (k1 > nchunks) k1 = nchunks;
#pragma unroll 8
    for (int k = g * rpg + pl; k < k1; k += FIN_PL) {
      a += ws[(long)k * stride_k + c];
      b += ws[(long)k * stride_k + off_q + c];
    }
  }
  ra[pl][cl] = a;
  rb[pl][cl] = b;
  __syncthreads();
  if (pl == 0 && c < C) {  // wave 0 alone stores the group row, so its own release covers it
    float ta = 0.f, tb = 0.f;
#pragma unroll
    for (int i = 0; i < FIN_PL; ++i) {
      ta += ra[i][cl];
      tb += rb[i][cl];
    }
    gws[(long)g * 2 * C + c] = ta;
    gws[(long)g * 2 * C + C + c] = tb;
  }
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(tickets + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
           (unsigned)(G - 1);
  }
  __syncthreads();
  if (!last) return;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    __hip_atomic_store(tickets + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  double sa = 0.0, sb = 0.0;
  if (c < C) {
    for (int k = pl; k < G; k += FIN_PL) {
      sa += gws[(long)k * 2 * C + c];
      sb += gws[(long)k * 2 * C + C + c];
    }
  }
  da[pl][cl] = sa;
  db[pl][cl] = sb;
  __syncthreads();
  if (pl == 0 && c < C) {
    double ta = 0.0, tb = 0.0;
#pragma unroll
    for (int i = 0; i < FIN_PL; ++i) {
      ta += da[i][cl];
      tb += db[i][cl];
    }
    F(c, ta, tb);
  }
}

template <bool RELU, bool DRES>
__global__ void __launch_bounds__(BLK) bn_bwd_apply_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y,
                                                          const uint8_t* __restrict__ mask,
                                                          const bf16_t* __restrict__ x, const float* __restrict__ coef,
                                                          bf16_t* __restrict__ dx, bf16_t* __restrict__ dres,
                                                          long M, int C, const Tiling tl) {
  const Tiling& t = tl;
  const int tx = threadIdx.x % t.TW, ty = threadIdx.x / t.TW;
  const int vc = blockIdx.x * t.TW + tx;
  if (vc >= t.CT) return;
  float A[8], B[8], D[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    A[j] = coef[vc * 8 + j];
    B[j] = coef[C + vc * 8 + j];
    D[j] = coef[2 * C + vc * 8 + j];
  }
  // contiguous row chunk per block, or (ilv) RP-row groups dealt round-robin so that the
  // blocks in flight sweep one contiguous span instead of ~nchunks far-apart streams
  const long step = t.ilv ? (long)gridDim.y * t.RP : t.RP;
  const long r0 = t.ilv ? (long)blockIdx.y * t.RP : (long)blockIdx.y * t.rows_per_chunk;
  long r1 = t.ilv ? M : r0 + t.rows_per_chunk;
  if (r1 > M) r1 = M;
  const long off0 = (long)vc * 8;
  for (long r = r0 + ty; r < r1; r += step) {
    const long o = r * C + off0;
    float d[8], xv[8];
    ld8bf(dy + o, d);
    ld8bf(x + o, xv);
    if (RELU) relu_gate(d, y, mask, r, o, t.CT, vc);
    if (DRES) st8bf(dres + o, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[j] = bn_bwd_affine(A[j], d[j], B[j], xv[j], D[j]);
    st8bf(dx + o, xv);
  }
}

}  // namespace

namespace {

// Per-stream ticket words of group_finalize_kernel (one per 64-channel column block;
// every launch leaves them at zero).  Streams get their own so concurrent BatchNorms on
// different streams never share a counter.
constexpr int MAX_TICKETS = 64;
unsigned* bn_tickets(hipStream_t s) {
  static std::mutex mu;
  static hipStream_t keys[16];
  static unsigned* slots[16];
  static int used = 0;
  std::lock_guard<std::mutex> lk(mu);
  for (int k = 0; k < used; ++k)
    if (keys[k] == s) return slots[k];
  if (used == 16) return nullptr;
  // no allocation inside a hipGraph capture: the two-launch path is captured instead
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  unsigned* t = nullptr;
  if (hipMalloc(&t, MAX_TICKETS * sizeof(unsigned)) != hipSuccess) return nullptr;
  if (hipMemsetAsync(t, 0, MAX_TICKETS * sizeof(unsigned), s) != hipSuccess) return nullptr;
  keys[used] = s;
  slots[used++] = t;
  return t;
}

bool merged_finalize() {  // CLOUD_AMD_BN_FIN_MERGED=0: separate group-reduce and finalize launches (A/B)
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CLOUD_AMD_BN_FIN_MERGED");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v != 0;
}

// Reduce [nchunks] partial rows (row k: a at ws[k*stride_k + c], b at +off_q) and run the
// per-channel finalize F: directly when the rows are few, else group-reduce into gws
// ([512][2][C]) and finalize -- one launch when the ticket path is available, two otherwise.
template <class FIN, class FinKernel>
int reduce_finalize(const float* ws, int nchunks, long stride_k, long off_q, int C, float* gws, const FIN& F,
                    FinKernel fin_kernel, hipStream_t s) {
  if (nchunks > 64 && gws) {
    unsigned* tk = (merged_finalize() && ca_cdiv(C, 64) <= MAX_TICKETS) ? bn_tickets(s) : nullptr;
    const int rpg = fin_rpg();
    if (tk && ca_cdiv(nchunks, rpg) <= 512) {  // (gws holds 512 group rows)
      const dim3 g1(ca_cdiv(C, 64), ca_cdiv(nchunks, rpg));
      group_finalize_kernel<FIN><<<g1, 64 * FIN_PL, 0, s>>>(ws, nchunks, stride_k, off_q, C, rpg, gws, tk, F);
      CA_LAUNCH_CHECK();
      return 0;
    }
    const int G = group_count(nchunks);
    const dim3 grid(ca_cdiv(C, 64), G);
    chunk_group_reduce_kernel<<<grid, 256, 0, s>>>(ws, nchunks, stride_k, off_q, C, gws);
    CA_LAUNCH_CHECK();
    fin_kernel<<<ca_cdiv(C, 4), 256, 0, s>>>(gws, G, 2L * C, (long)C, C, F);
  } else {
    fin_kernel<<<ca_cdiv(C, 4), 256, 0, s>>>(ws, nchunks, stride_k, off_q, C, F);
  }
  CA_LAUNCH_CHECK();
  return 0;
}

__global__ void bn_bwd_finalize_c_kernel(const float* __restrict__ ws, int nchunks, long stride_k, long off_q, int,
                                         const BwdFin F) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= F.C) return;
  double sd, sdx;
  wave_chunk_sum(ws, nchunks, stride_k, off_q, c, sd, sdx);
  if ((threadIdx.x & 63) != 0) return;
  F(c, sd, sdx);
}

}  // namespace

extern "C" {

// Workspace floats needed by the stats / bwd-reduce kernels: 2 * nchunks * C.
long ca_bn_workspace_floats(long M, int C) {
  Tiling t = make_tiling(M, C);
  return 2L * t.nchunks * C + 2L * 64 * C;
}

int ca_bn_fwd(const bf16_t* x, const bf16_t* res, bf16_t* y, long M, int C,
              const float* gamma, const float* beta, float eps, float momentum,
              float* run_mean, float* run_var, float* save_mean, float* save_rstd,
              float* scale_shift /* [2C] */, float* ws, int relu, uint8_t* mask, hipStream_t s) {
  if (C % 8 != 0) return -1;
  Tiling t = make_tiling(M, C);
  dim3 grid(t.ncol, t.nchunks);
  const Tiling ta = apply_tiling(M, C);
  const dim3 agrid(ta.ncol, ta.nchunks);
  bn_stats_kernel<<<grid, BLK, 0, s>>>(x, M, C, ws);
  CA_LAUNCH_CHECK();
  const FwdFin F{M, gamma, beta, eps, momentum, run_mean, run_var, save_mean, save_rstd, scale_shift, scale_shift + C};
  reduce_finalize(ws, t.nchunks, (long)C, (long)t.nchunks * C, C, nullptr, F, bn_fwd_finalize_kernel, s);
  if (relu && res) bn_apply_kernel<true, true><<<agrid, BLK, 0, s>>>(x, res, scale_shift, scale_shift + C, y, mask, M, C, ta);
  else if (relu) bn_apply_kernel<true, false><<<agrid, BLK, 0, s>>>(x, res, scale_shift, scale_shift + C, y, mask, M, C, ta);
  else if (res) bn_apply_kernel<false, true><<<agrid, BLK, 0, s>>>(x, res, scale_shift, scale_shift + C, y, mask, M, C, ta);
  else bn_apply_kernel<false, false><<<agrid, BLK, 0, s>>>(x, res, scale_shift, scale_shift + C, y, mask, M, C, ta);
  CA_LAUNCH_CHECK();
  return 0;
}

// Training forward from statistics partials produced by a GEMM/conv epilogue:
// partials[k][0][c] = sum, partials[k][1][c] = sum of squares over tile k.
int ca_bn_fwd_partials(const bf16_t* x, const bf16_t* res, bf16_t* y, long M, int C, const float* partials,
                       int nparts, const float* gamma, const float* beta, float eps, float momentum,
                       float* run_mean, float* run_var, float* save_mean, float* save_rstd,
                       float* scale_shift, int relu, uint8_t* mask, float* gws /* [512][2][C] or null */,
                       hipStream_t s) {
  if (C % 8 != 0) return -1;
  Tiling t = make_tiling(M, C);
  dim3 grid(t.ncol, t.nchunks);
  const Tiling ta = apply_tiling(M, C);
  const dim3 agrid(ta.ncol, ta.nchunks);
  const FwdFin F{M, gamma, beta, eps, momentum, run_mean, run_var, save_mean, save_rstd, scale_shift, scale_shift + C};
  reduce_finalize(partials, nparts, 2L * C, (long)C, C, gws, F, bn_fwd_finalize_kernel, s);
  if (relu && res) bn_apply_kernel<true, true><<<agrid, BLK, 0, s>>>(x, res, scale_shift, scale_shift + C, y, mask, M, C, ta);
  else if (relu) bn_apply_kernel<true, false><<<agrid, BLK, 0, s>>>(x, res, scale_shift, scale_shift + C, y, mask, M, C, ta);
  else if (res) bn_apply_kernel<false, true><<<agrid, BLK, 0, s>>>(x, res, scale_shift, scale_shift + C, y, mask, M, C, ta);
  else bn_apply_kernel<false, false><<<agrid, BLK, 0, s>>>(x, res, scale_shift, scale_shift + C, y, mask, M, C, ta);
  CA_LAUNCH_CHECK();
  return 0;
}

// ca_bn_fwd_partials, extended: y == null -> statistics / finalize only (scale_shift,
// save_*, running stats; no apply pass); res_ss != null -> the residual `res` is the input
// of another BatchNorm with that [scale | shift] (y = act(BN(x) + BN'(res)), see
// bn_apply_resbn_kernel).
int ca_bn_fwd_partials_ex(const bf16_t* x, const bf16_t* res, const float* res_ss, bf16_t* y, long M, int C,
                          const float* partials, int nparts, const float* gamma, const float* beta, float eps,
                          float momentum, float* run_mean, float* run_var, float* save_mean, float* save_rstd,
                          float* scale_shift, int relu, uint8_t* mask, float* gws, hipStream_t s) {
  if (C % 8 != 0 || (res_ss && !res)) return -1;
  if (y && !res_ss)
    return ca_bn_fwd_partials(x, res, y, M, C, partials, nparts, gamma, beta, eps, momentum, run_mean, run_var,
                              save_mean, save_rstd, scale_shift, relu, mask, gws, s);
  Tiling t = make_tiling(M, C);
  dim3 grid(t.ncol, t.nchunks);
  const Tiling ta = apply_tiling(M, C);
  const dim3 agrid(ta.ncol, ta.nchunks);
  const FwdFin F{M, gamma, beta, eps, momentum, run_mean, run_var, save_mean, save_rstd, scale_shift, scale_shift + C};
  reduce_finalize(partials, nparts, 2L * C, (long)C, C, gws, F, bn_fwd_finalize_kernel, s);
  if (!y) return 0;
  if (relu)
    bn_apply_resbn_kernel<true><<<agrid, BLK, 0, s>>>(x, res, scale_shift, scale_shift + C, res_ss, res_ss + C, y,
                                                     mask, M, C, ta);
  else
    bn_apply_resbn_kernel<false><<<agrid, BLK, 0, s>>>(x, res, scale_shift, scale_shift + C, res_ss, res_ss + C, y,
                                                      mask, M, C, ta);
  CA_LAUNCH_CHECK();
  return 0;
}

// Inference / frozen-stat apply with precomputed scale/shift.
int ca_bn_apply(const bf16_t* x, const bf16_t* res, bf16_t* y, long M, int C,
                const float* scale_shift, int relu, hipStream_t s) {
  uint8_t* mask = nullptr;
  if (C % 8 != 0) return -1;
  Tiling t = make_tiling(M, C);
  dim3 grid(t.ncol, t.nchunks);
  const Tiling ta = apply_tiling(M, C);
  const dim3 agrid(ta.ncol, ta.nchunks);
  if (relu && res) bn_apply_kernel<true, true><<<agrid, BLK, 0, s>>>(x, res, scale_shift, scale_shift + C, y, mask, M, C, ta);
  else if (relu) bn_apply_kernel<true, false><<<agrid, BLK, 0, s>>>(x, res, scale_shift, scale_shift + C, y, mask, M, C, ta);
  else if (res) bn_apply_kernel<false, true><<<agrid, BLK, 0, s>>>(x, res, scale_shift, scale_shift + C, y, mask, M, C, ta);
  else bn_apply_kernel<false, false><<<agrid, BLK, 0, s>>>(x, res, scale_shift, scale_shift + C, y, mask, M, C, ta);
  CA_LAUNCH_CHECK();
  return 0;
}

// y may be null when `mask` (the forward's ReLU bitmask) is given.
int ca_bn_bwd(const bf16_t* dy, const bf16_t* y, const uint8_t* mask, const bf16_t* x, long M, int C,
              const float* gamma, const float* save_mean, const float* save_rstd,
              bf16_t* dx, bf16_t* dres, float* dgamma, float* dbeta,
              float* coef /* [3C] */, float* ws, int relu, hipStream_t s) {
  if (C % 8 != 0) return -1;
  const int accum = (relu >> 1) & 1;  // flags: bit0 relu, bit1 accumulate dgamma/dbeta
  relu &= 1;
  Tiling t = make_tiling(M, C);
  dim3 grid(t.ncol, t.nchunks);
  const Tiling ta = apply_tiling(M, C);
  const dim3 agrid(ta.ncol, ta.nchunks);
  if (relu) bn_bwd_reduce_kernel<true><<<grid, BLK, 0, s>>>(dy, y, mask, x, save_mean, save_rstd, M, C, ws);
  else bn_bwd_reduce_kernel<false><<<grid, BLK, 0, s>>>(dy, y, mask, x, save_mean, save_rstd, M, C, ws);
  CA_LAUNCH_CHECK();
  // ws = [nchunks][C] (a) ++ [nchunks][C] (b); group-reduce into the tail of ws
  float* gws = ws + 2L * t.nchunks * C;
  const BwdFin F{M, C, gamma, save_mean, save_rstd, dgamma, dbeta, coef, accum, 0};
  if (t.nchunks > 64)
    reduce_finalize(ws, t.nchunks, (long)C, (long)t.nchunks * C, C, gws, F, bn_bwd_finalize_c_kernel, s);
  else
    reduce_finalize(ws, t.nchunks, (long)C, (long)t.nchunks * C, C, nullptr, F, bn_bwd_finalize_c_kernel, s);
  if (relu && dres) bn_bwd_apply_kernel<true, true><<<agrid, BLK, 0, s>>>(dy, y, mask, x, coef, dx, dres, M, C, ta);
  else if (relu) bn_bwd_apply_kernel<true, false><<<agrid, BLK, 0, s>>>(dy, y, mask, x, coef, dx, dres, M, C, ta);
  else if (dres) bn_bwd_apply_kernel<false, true><<<agrid, BLK, 0, s>>>(dy, y, mask, x, coef, dx, dres, M, C, ta);
  else bn_bwd_apply_kernel<false, false><<<agrid, BLK, 0, s>>>(dy, y, mask, x, coef, dx, dres, M, C, ta);
  CA_LAUNCH_CHECK();
  return 0;
}

// Backward from the [nparts][2][C] partials [sum dz | sum dz*x] written by a dgrad
// GEMM's BN-statistics epilogue (ca_gemm_bf16_bnstats / ca_conv_dgrad_bnstats): no
// reduction pass over dy and x; finalize (+group reduce) then the apply pass -- or, with
// dx == null, the finalize only (dgamma / dbeta and the [A | B | D] coefficients).
int ca_bn_bwd_partials(const bf16_t* dy, const bf16_t* y, const uint8_t* mask, const bf16_t* x, long M, int C,
                       const float* partials, int nparts, const float* gamma, const float* save_mean,
                       const float* save_rstd, bf16_t* dx, bf16_t* dres, float* dgamma, float* dbeta,
                       float* coef /* [3C] */, float* gws /* [512][2][C] */, int relu, hipStream_t s) {
  if (C % 8 != 0 || (nparts > 64 && !gws)) return -1;
  const int accum = (relu >> 1) & 1;
  relu &= 1;
  Tiling t = make_tiling(M, C);
  dim3 grid(t.ncol, t.nchunks);
  const Tiling ta = apply_tiling(M, C);
  const dim3 agrid(ta.ncol, ta.nchunks);
  const BwdFin F{M, C, gamma, save_mean, save_rstd, dgamma, dbeta, coef, accum, 1};
  reduce_finalize(partials, nparts, 2L * C, (long)C, C, gws, F, bn_bwd_finalize_c_kernel, s);
  if (!dx) return 0;  // finalize only: the apply runs in the consuming GEMM's operand fetch (ca_gemm_xa)
  if (relu && dres) bn_bwd_apply_kernel<true, true><<<agrid, BLK, 0, s>>>(dy, y, mask, x, coef, dx, dres, M, C, ta);
  else if (relu) bn_bwd_apply_kernel<true, false><<<agrid, BLK, 0, s>>>(dy, y, mask, x, coef, dx, dres, M, C, ta);
  else if (dres) bn_bwd_apply_kernel<false, true><<<agrid, BLK, 0, s>>>(dy, y, mask, x, coef, dx, dres, M, C, ta);
  else bn_bwd_apply_kernel<false, false><<<agrid, BLK, 0, s>>>(dy, y, mask, x, coef, dx, dres, M, C, ta);
  CA_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
