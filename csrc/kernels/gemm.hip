// bf16 MFMA GEMM family for NHWC convolutions / dense layers (K1 in SURVEY.md 2.7).
//
//   C[M,N] (+)= A[M,K] * B[K,N]      bf16 in, fp32 accumulate
//
// Operand layouts (template flags):
//   A_KC = true : A stored [M][K] (K contiguous)      -- activations in forward
//   A_KC = false: A stored [K][M] (M contiguous)      -- dY^T in weight-gradient
//   B_KC = true : B stored [N][K] (K contiguous)      -- weights [Cout][Cin] in forward
//   B_KC = false: B stored [K][N] (N contiguous)      -- weights in dgrad, X in wgrad
// so forward (Y = X W^T), dgrad (dX = dY W) and wgrad (dW = dY^T X) of a 1x1
// NHWC convolution all read the tensors exactly as they lie in memory.
//
// Structure (CDNA4): v_mfma_f32_16x16x32_bf16, BK = 64, one workgroup =
// WM x WN waves (64 lanes each), register-staged global->LDS double buffering
// with one barrier per K step (issue next tile's 16-B loads before the MFMAs,
// write them to the other LDS buffer after).  K-contiguous tiles are read with
// ds_read_b128 from 16-B padded rows (conflict-free for 16 consecutive rows);
// M/N-contiguous tiles are read as MFMA fragments with the gfx950 transposed
// LDS read ds_read_b64_tr_b16 (two per fragment).  Block index -> tile mapping
// is XCD-aware (contiguous tile ranges per XCD so neighbouring tiles share an
// L2).  Split-K over grid.z writes fp32 partial slabs reduced by a second
// kernel (deterministic; no float atomics).
//
// Epilogues: (0) bf16 store, (1) fp32 partial slab store (split-K),
// (2) bf16 store + per-column sum / sum-of-squares partials of the stored
// bf16 values (fused BatchNorm statistics for the next BN layer).
#include "ca_common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s8v __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4v lds_s4v;

constexpr int BK = 64;
constexpr int PAD = 8;  // elements of padding per LDS row (16 B)

enum { EPI_BF16 = 0, EPI_F32_PARTIAL = 1, EPI_BF16_STATS = 2 };

struct GemmArgs {
  const bf16_t* A; long lda;
  const bf16_t* B; long ldb;
  void* C; long ldc;
  float* stats;        // EPI_BF16_STATS: [gridM][2][N]
  int M, N, K;
  int k_per_split;     // K range per grid.z slice (multiple of BK)
  long split_stride;   // EPI_F32_PARTIAL: elements between split slabs
};

// LDS tile geometry for an operand tile covering `R` rows of the output
// dimension (BM or BN) and BK of the reduction dimension.
template <int R, bool KC>
struct TileGeom {
  // KC: [R][BK+PAD]   non-KC: [BK][R+PAD]
  static constexpr int ROWS = KC ? R : BK;
  static constexpr int COLS = KC ? BK : R;
  static constexpr int LD = COLS + PAD;
  static constexpr int ELEMS = ROWS * LD;
  static constexpr int CHUNKS = ROWS * COLS / 8;  // 16-B chunks per tile
};

// Global -> registers: CPT chunks of 16 B per thread.
template <int R, bool KC, int NT>
struct Stager {
  using G = TileGeom<R, KC>;
  static constexpr int CPT = G::CHUNKS / NT;
  static_assert(G::CHUNKS % NT == 0, "tile chunks must divide threads");
  s8v regs[CPT];

  // base: element offset of the tile's (r0, k0) corner; bound: rows valid along R
  __device__ __forceinline__ void load(const bf16_t* __restrict__ p, long ld, int r0, int k0, int rlimit, int tid) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = tid + i * NT;
      const int row = c / (G::COLS / 8);
      const int col = (c % (G::COLS / 8)) * 8;
      bool ok;
      long off;
      if (KC) {  // row = r (output dim), col = k
        ok = (r0 + row) < rlimit;
        off = (long)(r0 + row) * ld + (k0 + col);
      } else {   // row = k, col = r
        ok = (r0 + col) < rlimit;
        off = (long)(k0 + row) * ld + (r0 + col);
      }
      if (ok) regs[i] = *reinterpret_cast<const s8v*>(p + off);
      else regs[i] = s8v{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  __device__ __forceinline__ void store(short* lds, int tid) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = tid + i * NT;
      const int row = c / (G::COLS / 8);
      const int col = (c % (G::COLS / 8)) * 8;
      *reinterpret_cast<s8v*>(lds + row * G::LD + col) = regs[i];
    }
  }
};

// MFMA 16x16x32 fragment: lane l holds X[r0 + (l&15)][k0 + 8*(l>>4) + j], j = 0..7
// where X is the operand in (output-dim, k) orientation.
template <int R, bool KC>
__device__ __forceinline__ bf16x8 read_frag(const short* lds, int r0, int k0, int lane) {
  using G = TileGeom<R, KC>;
  if constexpr (KC) {
    s8v v = *reinterpret_cast<const s8v*>(lds + (r0 + (lane & 15)) * G::LD + k0 + 8 * (lane >> 4));
    return __builtin_bit_cast(bf16x8, v);
  } else {
    // LDS is [k][r]; ds_read_b64_tr_b16: lane 4q+p of each 16-lane group addresses
    // row q, columns 4p..4p+3 of a 4x16 block; receives column (lane&15) of the 4 rows.
    const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
    const short* b0 = lds + (k0 + 8 * g + q) * G::LD + r0 + 4 * p;
    s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(b0));
    s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(b0 + 4 * G::LD));
    s8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// XCD-aware bijective remap of a linear block id (cdna_hip_programming.md 5.5 T1).
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  const int xcd = bid & 7, q = nblk >> 3, r = nblk & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

template <int BM, int BN, int WM, int WN, bool A_KC, bool B_KC, int EPI>
__global__ void __launch_bounds__(WM * WN * 64) gemm_kernel(GemmArgs args) {
  constexpr int NT = WM * WN * 64;
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;
  using GA = TileGeom<BM, A_KC>;
  using GB = TileGeom<BN, B_KC>;
  constexpr int STAGE = GA::ELEMS + GB::ELEMS;
  constexpr int EPI_LD = BN + PAD;
  constexpr int SMEM = (2 * STAGE > BM * EPI_LD ? 2 * STAGE : BM * EPI_LD);
  __shared__ __attribute__((aligned(16))) short smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_m = (args.M + BM - 1) / BM, tiles_n = (args.N + BN - 1) / BN;
  const int nblk = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nblk);
  // N-fastest within an XCD's contiguous range: consecutive blocks share the A panel
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = blockIdx.z * args.k_per_split;
  int kend = kbeg + args.k_per_split;
  if (kend > args.K) kend = args.K;
  const int nk = (kend - kbeg) / BK;

  Stager<BM, A_KC, NT> sa;
  Stager<BN, B_KC, NT> sb;
  f4v acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    sa.load(args.A, args.lda, m0, kbeg, args.M, tid);
    sb.load(args.B, args.ldb, n0, kbeg, args.N, tid);
    sa.store(smem, tid);
    sb.store(smem + GA::ELEMS, tid);
  }
  __syncthreads();
  int cur = 0;
  for (int t = 0; t < nk; ++t) {
    const bool more = (t + 1) < nk;
    if (more) {
      const int k1 = kbeg + (t + 1) * BK;
      sa.load(args.A, args.lda, m0, k1, args.M, tid);
      sb.load(args.B, args.ldb, n0, k1, args.N, tid);
    }
    const short* As = smem + cur * STAGE;
    const short* Bs = As + GA::ELEMS;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = read_frag<BM, A_KC>(As, wm * (BM / WM) + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = read_frag<BN, B_KC>(Bs, wn * (BN / WN) + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      short* nxt = smem + (cur ^ 1) * STAGE;
      sa.store(nxt, tid);
      sb.store(nxt + GA::ELEMS, tid);
    }
    __syncthreads();
    cur ^= 1;
  }

  // C mapping of mfma_f32_16x16x32: col = lane&15, row = (lane>>4)*4 + r
  const int rbase = wm * (BM / WM) + (lane >> 4) * 4;
  const int cbase = wn * (BN / WN) + (lane & 15);
  if constexpr (EPI == EPI_F32_PARTIAL) {
    float* Cp = reinterpret_cast<float*>(args.C) + (long)blockIdx.z * args.split_stride;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int gm = m0 + rbase + i * 16 + r, gn = n0 + cbase + j * 16;
          if (gm < args.M && gn < args.N) Cp[(long)gm * args.ldc + gn] = acc[i][j][r];
        }
    return;
  } else {
    // Stage the bf16 tile through LDS, then 16-B coalesced stores.
    short* Cs = smem;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Cs[(rbase + i * 16 + r) * EPI_LD + cbase + j * 16] = (short)f2bf(acc[i][j][r]);
    __syncthreads();
    bf16_t* Cg = reinterpret_cast<bf16_t*>(args.C);
    constexpr int CH = BM * BN / 8;
#pragma unroll
    for (int c = tid; c < CH; c += NT) {
      const int row = c / (BN / 8), col = (c % (BN / 8)) * 8;
      const int gm = m0 + row, gn = n0 + col;
      if (gm < args.M && gn < args.N)
        *reinterpret_cast<s8v*>(Cg + (long)gm * args.ldc + gn) = *reinterpret_cast<const s8v*>(Cs + row * EPI_LD + col);
    }
    if constexpr (EPI == EPI_BF16_STATS) {
      // column sums over the valid rows of this tile; NT/BN threads per column
      constexpr int TPC = NT / BN;
      const int col = tid % BN, part = tid / BN;
      float s = 0.f, q = 0.f;
      int rows = args.M - m0;
      if (rows > BM) rows = BM;
      for (int r = part; r < rows; r += TPC) {
        const float v = bf2f((bf16_t)Cs[r * EPI_LD + col]);
        s += v;
        q += v * v;
      }
      __syncthreads();
      // reuse the (now consumed) staging region beyond the C tile for the reduction
      float* sred = reinterpret_cast<float*>(smem);
      sred[part * BN + col] = s;
      sred[(TPC + part) * BN + col] = q;
      __syncthreads();
      if (part == 0 && n0 + col < args.N) {
        float ts = 0.f, tq = 0.f;
#pragma unroll
        for (int pp = 0; pp < TPC; ++pp) {
          ts += sred[pp * BN + col];
          tq += sred[(TPC + pp) * BN + col];
        }
        float* st = args.stats + (long)tm * 2 * args.N;
        st[n0 + col] = ts;
        st[args.N + n0 + col] = tq;
      }
    }
  }
}

// Sum S fp32 slabs [S][M][N] -> out (bf16 or fp32), optionally accumulating.
template <bool OUT_BF16>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ ws, int S, long MN,
                                                           void* __restrict__ out, float beta) {
  const long n4 = MN / 4;
  for (long v = (long)blockIdx.x * blockDim.x + threadIdx.x; v < n4; v += (long)gridDim.x * blockDim.x) {
    f4v acc = *reinterpret_cast<const f4v*>(ws + v * 4);
    for (int s = 1; s < S; ++s) acc += *reinterpret_cast<const f4v*>(ws + (long)s * MN + v * 4);
    if (OUT_BF16) {
      bf16_t* o = reinterpret_cast<bf16_t*>(out) + v * 4;
      if (beta != 0.f) {
        us4 old = *reinterpret_cast<const us4*>(o);
        for (int j = 0; j < 4; ++j) acc[j] += beta * bf2f(old[j]);
      }
      us4 r;
      for (int j = 0; j < 4; ++j) r[j] = f2bf(acc[j]);
      *reinterpret_cast<us4*>(o) = r;
    } else {
      float* o = reinterpret_cast<float*>(out) + v * 4;
      if (beta != 0.f) acc += beta * *reinterpret_cast<const f4v*>(o);
      *reinterpret_cast<f4v*>(o) = acc;
    }
  }
}

template <int BM, int BN, int WM, int WN, bool A_KC, bool B_KC, int EPI>
int launch(const GemmArgs& a, int splits, hipStream_t s) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  dim3 grid(tiles, 1, splits);
  gemm_kernel<BM, BN, WM, WN, A_KC, B_KC, EPI><<<grid, WM * WN * 64, 0, s>>>(a);
  CA_LAUNCH_CHECK();
  return 0;
}

// layout code: 0 = NT (A KC, B KC), 1 = NN (A KC, B NC), 2 = TN (A MC, B NC)
template <int EPI>
int dispatch(int layout, const GemmArgs& a, int splits, hipStream_t s) {
  const bool small_n = a.N <= 64;
  switch (layout) {
    case 0:
      return small_n ? launch<128, 64, 2, 2, true, true, EPI>(a, splits, s)
                     : launch<128, 128, 2, 2, true, true, EPI>(a, splits, s);
    case 1:
      return small_n ? launch<128, 64, 2, 2, true, false, EPI>(a, splits, s)
                     : launch<128, 128, 2, 2, true, false, EPI>(a, splits, s);
    case 2:
      return small_n ? launch<128, 64, 2, 2, false, false, EPI>(a, splits, s)
                     : launch<128, 128, 2, 2, false, false, EPI>(a, splits, s);
  }
  return -2;
}

}  // namespace

extern "C" {

// C[M,N] = A*B (bf16 out).  layout: 0 NT, 1 NN, 2 TN (see header).  stats != null
// -> also write per-128-row-tile column sum/sumsq partials [ceil(M/128)][2][N].
int ca_gemm_bf16(int layout, const bf16_t* A, long lda, const bf16_t* B, long ldb, bf16_t* C, long ldc,
                 int M, int N, int K, float* stats, hipStream_t s) {
  if (K % BK != 0 || N % 8 != 0 || (layout == 2 && M % 8 != 0)) return -1;
  GemmArgs a{A, lda, B, ldb, C, ldc, stats, M, N, K, K, 0};
  return stats ? dispatch<EPI_BF16_STATS>(layout, a, 1, s) : dispatch<EPI_BF16>(layout, a, 1, s);
}

// Split-K GEMM into fp32 slabs ws[splits][M][N] followed by a reduction into
// `out` (bf16 if out_bf16 else fp32), out = sum + beta*out.
int ca_gemm_splitk(int layout, const bf16_t* A, long lda, const bf16_t* B, long ldb, void* out, int out_bf16,
                   float beta, int M, int N, int K, int splits, float* ws, hipStream_t s) {
  if (K % BK != 0 || N % 8 != 0 || (layout == 2 && M % 8 != 0)) return -1;
  int kps = (K / splits + BK - 1) / BK * BK;
  splits = (K + kps - 1) / kps;
  GemmArgs a{A, lda, B, ldb, ws, (long)N, nullptr, M, N, K, kps, (long)M * N};
  int rc = dispatch<EPI_F32_PARTIAL>(layout, a, splits, s);
  if (rc) return rc;
  const long MN = (long)M * N;
  if (MN % 4) return -3;
  const int grid = ca_stream_grid(MN / 4, 256);
  if (out_bf16) splitk_reduce_kernel<true><<<grid, 256, 0, s>>>(ws, splits, MN, out, beta);
  else splitk_reduce_kernel<false><<<grid, 256, 0, s>>>(ws, splits, MN, out, beta);
  CA_LAUNCH_CHECK();
  return 0;
}

int ca_gemm_splitk_effective(int K, int splits) {
  int kps = (K / splits + BK - 1) / BK * BK;
  return (K + kps - 1) / kps;
}

}  // extern "C"
