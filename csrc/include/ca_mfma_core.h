// Shared MFMA GEMM core for cloud_amd's dense and implicit-GEMM convolution
// kernels (gfx950 / CDNA4).
//
//   C[M,N] = sum_k A(m,k) * B(k,n)      bf16 operands, fp32 accumulation
//
// The core is parameterised by two *loader* policies (how a 16-B chunk of the
// A or B tile is fetched from global memory: dense row-major, or gathered from
// an NHWC activation for implicit-GEMM convolution) and an epilogue mode.
//
//  * MFMA: v_mfma_f32_16x16x32_bf16; a workgroup = WM x WN waves of 64 lanes.
//  * BK = 64; register-staged global->LDS double buffering, one barrier per K
//    step: the next tile's 16-B global loads are issued before this tile's
//    MFMAs and written to the other LDS buffer after them.
//  * K-contiguous tiles ("KC") live in LDS as [rows][64+8] and feed MFMA with
//    ds_read_b128 (16-B padded rows: conflict-free for 16 consecutive rows);
//    M/N-contiguous tiles ("NC") live as [64][rows+8] and feed MFMA through the
//    gfx950 transposed read ds_read_b64_tr_b16 (two per fragment).
//  * blockIdx -> tile mapping is XCD-aware and bijective (contiguous tile
//    ranges per XCD share an L2).
//  * Split-K over grid.z writes fp32 slabs (deterministic reduce kernel).
#pragma once
#include "ca_common.h"

namespace ca {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s8v __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4v lds_s4v;

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int BK = 64;
constexpr int PAD = 8;

constexpr uint32_t BUF_CAP = 0x7fffffc0u;  // byte range of one buffer resource (offsets stay < 2 GiB)

__device__ __forceinline__ uint32_t buf_span(long bytes) {
  return bytes <= 0 ? 0u : (bytes >= (long)BUF_CAP ? BUF_CAP : (uint32_t)bytes);
}

// EPI_BF16_BN: EPI_BF16 plus the BN-backward statistics (CoreParams::bnz);
// EPI_BF16_ST: EPI_BF16 plus the BN-forward statistics [sum | sum of squares] of the
// stored values, accumulated in registers by the storing thread.  Separate
// instantiations, so the plain bf16 epilogue carries none of their registers.
// EPI_BF16_BNR: EPI_BF16_BN that also honours CoreParams::res_src / res_mask (the
// plain bf16 epilogue always does; the BN-statistics one only in this instantiation).
// EPI_BF16_BNR2: EPI_BF16_BNR that also sums g * z2 for a second BatchNorm fed by the same
// gradient (CoreParams::bnz2 / stats2: the projection shortcut's BN, whose input is the
// shortcut convolution output and whose output gradient is the same gated block gradient).
enum Epi { EPI_BF16 = 0, EPI_F32_PARTIAL = 1, EPI_BF16_BN = 2, EPI_BF16_ST = 3, EPI_BF16_BNR = 4, EPI_BF16_BNR2 = 5 };

// Fast unsigned division by a runtime constant (n < 2^31): q = (umulhi(n, m) + n) >> s.
struct FastDiv {
  uint32_t d, m, s;
};
static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while (s < 32 && (1u << s) < d) ++s;
  const uint64_t one = 1;
  f.m = (uint32_t)(((one << 32) * ((one << s) - d)) / d + 1);
  f.s = s;
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (__umulhi(n, f.m) + n) >> f.s;
}

// Everything any loader / epilogue may need (one kernel-argument struct).
struct CoreParams {
  const bf16_t* A; long lda;
  const bf16_t* B; long ldb;
  void* C; long ldc;
  float* stats;          // optional: per-M-tile column [sum | sumsq] partials [tiles_m][2][N]
  // BN-backward statistics epilogue (dgrad GEMMs whose output dy feeds a BatchNorm(+ReLU)
  // backward): with bnz set, `stats` receives per-tile column [sum g | sum g*z] where
  // g = dy * relu'(mask) and z is the BN input (same [rows][ldc] layout as C).
  const bf16_t* bnz;
  const uint8_t* bnmask;  // ReLU bitmask [rows][N/8] (bit j = channel 8c+j active) or null
  const bf16_t* bnz2;     // EPI_BF16_BNR2: second BN input (same layout as bnz) ...
  float* stats2;          // ... and its partials [tiles][2][N] = [sum g | sum g*z2]
  // beta source other than C: C = acc + beta * relu'(res_mask) * res_src (same [rows][ldc]
  // layout as C) -- a residual gradient gated on the fly instead of materialised first
  const bf16_t* res_src;
  const uint8_t* res_mask;
  float beta;            // C = acc + beta * C_old (bf16 epilogue)
  int M, N, K;
  int k_per_split;
  long split_stride;
  // convolution geometry (NHWC input [Nb,H,W,Cin], output [Nb,OH,OW,Cout], weights [Cout][KH][KW][Cin])
  int Nb, H, W, Cin, OH, OW, Cout, KH, KW, sh, sw, ph, pw;
  FastDiv div_ow, div_oh, div_w, div_h, div_cin, div_cout, div_kw;
  int cin_tile, cout_tile;  // Cin % BK == 0 / Cout % BK == 0: a K tile never straddles two taps
  // dense-layer epilogue (bf16 path): C = act(acc + bias) with the pre-activation
  // optionally kept (preact), or, in the backward, C = acc * act'(dact_src).
  const float* bias;      // [N] fp32 or null
  int act;                // ACT_* below
  bf16_t* preact;         // [M][ld_aux] or null
  const bf16_t* dact_src; // [M][ld_aux] or null (backward: multiply by act'(src))
  long ld_aux;
  // strided-conv dgrad by output-parity class (conv.hip): GEMM row m = (n, qy, qx) of
  // the class is stored at input pixel (n, s*qy + py, s*qx + px); taps kh = kh0 + s*th.
  int rowmap;
  int dg_py, dg_px, dg_kh0, dg_kw0, dg_nh, dg_nw, dg_dy0, dg_dx0, Hq, Wq;
  FastDiv div_wq, div_hq, div_nw;
  int split_xcd;  // split-K grids: deal (split, tile) ranges to XCDs split-major (blk_pos)
  int prw_chunks; // persistent resident-weight core: column chunks of BN (0 / 1 = the whole N resident)
  unsigned long long* stamps;  // diagnostic builds only (in-kernel s_memtime stamps)
  // sparse beta source: with bpar_s > 1 the old C (output rows = NHWC pixels of an
  // [*, H, W] image, W = div_bpw.d, H = div_bph.d) holds values only at pixels whose h and w
  // are multiples of bpar_s -- the others are implicit zeros, never read (a strided 1x1
  // convolution's input gradient, written for its one non-empty parity class only)
  int bpar_s;
  FastDiv div_bpw, div_bph;
};

// whether the beta-accumulate source of output row `orow` is stored (see CoreParams::bpar_s)
__device__ __forceinline__ bool beta_row_stored(const CoreParams& P, long orow) {
  if (P.bpar_s <= 1) return true;
  const uint32_t t = fdiv((uint32_t)orow, P.div_bpw);
  const int w = (int)((uint32_t)orow - t * P.div_bpw.d);
  const uint32_t t2 = fdiv(t, P.div_bph);
  const int h = (int)(t - t2 * P.div_bph.d);
  return (h % P.bpar_s) == 0 && (w % P.bpar_s) == 0;
}

// output row of GEMM row gm (identity unless the parity-class row map is on)
__device__ __forceinline__ long out_row(const CoreParams& P, int gm) {
  if (!P.rowmap) return gm;
  const uint32_t t = fdiv((uint32_t)gm, P.div_wq);
  const int qx = gm - (int)t * P.Wq;
  const uint32_t n = fdiv(t, P.div_hq);
  const int qy = (int)t - (int)n * P.Hq;
  return ((long)n * P.H + P.sh * qy + P.dg_py) * P.W + P.sw * qx + P.dg_px;
}

enum Act { ACT_NONE = 0, ACT_GELU = 1, ACT_RELU = 2, ACT_TANH = 3, ACT_GELU_TANH = 4, ACT_ELU = 5 };

// Phi(x) = 0.5 (1 + erf(x / sqrt 2)) for the erf-GELU epilogues, without erff: erfc(z) =
// t exp(-z^2 + P(t)), t = 1 / (1 + z / 2) (the Chebyshev-fitted form with fractional error
// < 1.2e-7 over all z, Numerical Recipes "erfcc"), log2(e) folded into P so the exponential
// is one v_exp_f32.  1 rcp + 1 exp + 11 FMA-class ops per element against ocml erff's two
// branchy polynomials.  Measured in the BERT step (docs/performance.md, "BERT step, round
// 3"): FFN1 forward 65.0 -> 64.9 us, FFN2 input-gradient with GELU' 74 -> 72 us -- those
// epilogues are bound by their 100 MB of stores, not by this arithmetic.
__device__ __forceinline__ float gelu_cdf(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, z, 1.f));
  float q = fmaf(t, 2.465172979e-01f, -1.186114945e+00f);
  q = fmaf(t, q, 2.147474464e+00f);
  q = fmaf(t, q, -1.637753152e+00f);
  q = fmaf(t, q, 4.023215817e-01f);
  q = fmaf(t, q, -2.687568603e-01f);
  q = fmaf(t, q, 1.396300565e-01f);
  q = fmaf(t, q, 5.397006155e-01f);
  q = fmaf(t, q, 1.442729204e+00f);
  q = fmaf(t, q, -1.825748218e+00f);
  const float h = 0.5f * t * __builtin_amdgcn_exp2f(fmaf(x, x * -0.72134752044448170f, q));  // erfc(z) / 2
  return x >= 0.f ? 1.f - h : h;
}

// Two elements at a time on packed-FP32 math (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32: two
// lanes' worth of FMAs per instruction; rcp / exp stay per element).  Same formula as gelu_cdf.
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v gelu_cdf2(f2v x) {
  const f2v z = __builtin_elementwise_abs(x) * 0.70710678118654752f;
  const f2v d = __builtin_elementwise_fma(f2v{0.5f, 0.5f}, z, f2v{1.f, 1.f});
  const f2v t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f2v q = __builtin_elementwise_fma(t, f2v{2.465172979e-01f, 2.465172979e-01f}, f2v{-1.186114945e+00f, -1.186114945e+00f});
  q = __builtin_elementwise_fma(t, q, f2v{2.147474464e+00f, 2.147474464e+00f});
  q = __builtin_elementwise_fma(t, q, f2v{-1.637753152e+00f, -1.637753152e+00f});
  q = __builtin_elementwise_fma(t, q, f2v{4.023215817e-01f, 4.023215817e-01f});
  q = __builtin_elementwise_fma(t, q, f2v{-2.687568603e-01f, -2.687568603e-01f});
  q = __builtin_elementwise_fma(t, q, f2v{1.396300565e-01f, 1.396300565e-01f});
  q = __builtin_elementwise_fma(t, q, f2v{5.397006155e-01f, 5.397006155e-01f});
  q = __builtin_elementwise_fma(t, q, f2v{1.442729204e+00f, 1.442729204e+00f});
  q = __builtin_elementwise_fma(t, q, f2v{-1.825748218e+00f, -1.825748218e+00f});
  const f2v e = __builtin_elementwise_fma(x, x * -0.72134752044448170f, q);
  const f2v h = 0.5f * t * f2v{__builtin_amdgcn_exp2f(e.x), __builtin_amdgcn_exp2f(e.y)};
  return f2v{x.x >= 0.f ? 1.f - h.x : h.x, x.y >= 0.f ? 1.f - h.y : h.y};
}

// GELU(x) / v * GELU'(x) on an 8-column bf16 chunk, two elements per packed step
__device__ __forceinline__ void gelu8(s8v& v) {
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    const f2v x = {bf2f((bf16_t)v[j]), bf2f((bf16_t)v[j + 1])};
    const f2v y = x * gelu_cdf2(x);
    v[j] = (short)f2bf(y.x);
    v[j + 1] = (short)f2bf(y.y);
  }
}
__device__ __forceinline__ void gelu_grad_mul8(s8v& v, const s8v& src) {
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    const f2v x = {bf2f((bf16_t)src[j]), bf2f((bf16_t)src[j + 1])};
    const f2v e = x * x * -0.72134752044448170f;
    const f2v d = __builtin_elementwise_fma(x * 0.3989422804014327f,
                                            f2v{__builtin_amdgcn_exp2f(e.x), __builtin_amdgcn_exp2f(e.y)}, gelu_cdf2(x));
    v[j] = (short)f2bf(bf2f((bf16_t)v[j]) * d.x);
    v[j + 1] = (short)f2bf(bf2f((bf16_t)v[j + 1]) * d.y);
  }
}

__device__ __forceinline__ float act_fwd(int act, float x) {
  switch (act) {
    case ACT_GELU: return x * gelu_cdf(x);
    case ACT_RELU: return x > 0.f ? x : 0.f;
    case ACT_TANH: return tanhf(x);
    case ACT_GELU_TANH: {
      const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
      return 0.5f * x * (1.f + tanhf(u));
    }
    case ACT_ELU: return x > 0.f ? x : expm1f(x);
  }
  return x;
}

// d act(x) / dx
__device__ __forceinline__ float act_grad(int act, float x) {
  switch (act) {
    case ACT_GELU:
      return fmaf(x * 0.3989422804014327f, __builtin_amdgcn_exp2f(x * x * -0.72134752044448170f), gelu_cdf(x));
    case ACT_RELU: return x > 0.f ? 1.f : 0.f;
    case ACT_TANH: {
      const float t = tanhf(x);
      return 1.f - t * t;
    }
    case ACT_GELU_TANH: {
      const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
      const float t = tanhf(u);
      return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * 0.7978845608028654f * (1.f + 3.f * 0.044715f * x * x);
    }
    case ACT_ELU: return x > 0.f ? 1.f : __expf(x);
  }
  return 1.f;
}

template <int R, bool KC>
struct TileGeom {
  static constexpr int ROWS = KC ? R : BK;
  static constexpr int COLS = KC ? BK : R;
  static constexpr int LD = COLS + PAD;
  static constexpr int ELEMS = ROWS * LD;
  static constexpr int CHUNKS = ROWS * COLS / 8;
};

template <int R, bool KC>
__device__ __forceinline__ void chunk_coords(int c, int& row, int& col) {
  using G = TileGeom<R, KC>;
  row = c / (G::COLS / 8);
  col = (c % (G::COLS / 8)) * 8;
}

template <int R, bool KC>
__device__ __forceinline__ bf16x8 read_frag(const short* lds, int r0, int k0, int lane) {
  using G = TileGeom<R, KC>;
  if constexpr (KC) {
    s8v v = *reinterpret_cast<const s8v*>(lds + (r0 + (lane & 15)) * G::LD + k0 + 8 * (lane >> 4));
    return __builtin_bit_cast(bf16x8, v);
  } else {
    const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
    const short* b0 = lds + (k0 + 8 * g + q) * G::LD + r0 + 4 * p;
    s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(b0));
    s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(b0 + 4 * G::LD));
    s8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  const int xcd = bid & 7, q = nblk >> 3, r = nblk & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// Block -> (output tile, K split).  Workgroups go to the 8 XCDs round-robin by linear
// id (x fastest, then z).  A split-K grid's tiles of one K chunk read the same K rows
// of both operands (a conv weight gradient's 5-9 column tiles all gather the same dY
// and X pixels), so with split_xcd each XCD gets a contiguous range of the
// split-major (split, tile) order and those re-reads hit its own L2 instead of
// being fetched once per XCD.  Without it the tiles of a split land on different XCDs.
// host: CLOUD_AMD_SPLIT_XCD=0 keeps the tile-only XCD remap on split-K grids (A/B runs)
inline int split_xcd_enabled() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CLOUD_AMD_SPLIT_XCD");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v;
}

struct BlkPos {
  int tile, split;
};
__device__ __forceinline__ BlkPos blk_pos(const CoreParams& P) {
  const int nt = gridDim.x;
  if (gridDim.z == 1 || !P.split_xcd) return {xcd_remap(blockIdx.x, nt), (int)blockIdx.z};
  const int lid = xcd_remap(blockIdx.x + nt * blockIdx.z, nt * gridDim.z);
  return {lid % nt, lid / nt};
}
__device__ __forceinline__ int blk_split(const CoreParams& P) { return blk_pos(P).split; }

__device__ __forceinline__ s8v zero8() { return s8v{0, 0, 0, 0, 0, 0, 0, 0}; }
__device__ __forceinline__ s8v ld16(const bf16_t* p) { return *reinterpret_cast<const s8v*>(p); }

// ---------------------------------------------------------------- loaders --
// A loader owns the CPT 16-B chunks a thread fetches per K tile.  Everything
// that depends only on the chunk's output-dim coordinate (row pointers, pixel
// decode) is computed ONCE in the constructor; load(i, k0) only adds the
// k-dependent part -- keeps the address VALU work out of the MFMA loop.
// KC loaders: chunk (row = output-dim offset, col = k offset).
// NC loaders: chunk (row = k offset, col = output-dim offset).

// Dense operand, K-contiguous: X[r][k] at p[r*ld + k].
template <int R, int CPT, int NT>
struct DenseKC {
  static constexpr bool KC = true;
  const bf16_t* rowp[CPT];
  int col[CPT];
  bool ok[CPT];
  int K;
  __device__ DenseKC(const CoreParams& P, bool isA, int r0, int tid) {
    const bf16_t* p = isA ? P.A : P.B;
    const long ld = isA ? P.lda : P.ldb;
    const int rlimit = isA ? P.M : P.N;
    K = P.K;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      int row, c;
      chunk_coords<R, true>(tid + i * NT, row, c);
      ok[i] = (r0 + row) < rlimit;
      rowp[i] = p + (long)(ok[i] ? r0 + row : 0) * ld;
      col[i] = c;
    }
  }
  __device__ __forceinline__ s8v load(int i, int k0) const {
    const int k = k0 + col[i];
    return (ok[i] && k < K) ? ld16(rowp[i] + k) : zero8();
  }
};

// Dense operand, output-dim contiguous: X[r][k] at p[k*ld + r].
template <int R, int CPT, int NT>
struct DenseNC {
  static constexpr bool KC = false;
  const bf16_t* colp[CPT];
  int row[CPT];
  bool ok[CPT];
  long ld;
  int K;
  __device__ DenseNC(const CoreParams& P, bool isA, int r0, int tid) {
    const bf16_t* p = isA ? P.A : P.B;
    ld = isA ? P.lda : P.ldb;
    const int rlimit = isA ? P.M : P.N;
    K = P.K;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      int r, c;
      chunk_coords<R, false>(tid + i * NT, r, c);
      ok[i] = (r0 + c) < rlimit;
      colp[i] = p + (ok[i] ? r0 + c : 0);
      row[i] = r;
    }
  }
  __device__ __forceinline__ s8v load(int i, int k0) const {
    const int k = k0 + row[i];
    return (ok[i] && k < K) ? ld16(colp[i] + (long)k * ld) : zero8();
  }
};

// LDS image of the bf16 C tile staged by the epilogue.  The accumulators are C^T
// fragments (see mfma_acc), so a lane owns 4 consecutive columns of one row and writes
// them as ONE 8-byte ds_write_b64 (16 per thread for a 128x128 tile, not 64 2-byte
// stores).  BN = 128: unpadded 256-B rows with the 8-column chunks XOR-swizzled by
// row & 15 -- the 16 rows one ds_write_b64 lane group touches land in 16 distinct
// 16-B bank slots, and the 16-B row reads of the store phase stay contiguous; the tile
// is exactly 32 KB (a 32-KB K stage keeps five 128x128 blocks per CU).  Other widths
// keep the padded layout (row stride 36 banks: conflict-free for the same pattern).
template <int BN>
struct EpiLayout {
  static constexpr bool SWZ = (BN >= 128) && (BN & (BN - 1)) == 0;  // XOR stays inside a power-of-two row
  static constexpr int LD = SWZ ? BN : BN + PAD;
  __device__ static __forceinline__ int idx(int row, int col) {
    return SWZ ? row * LD + (col ^ ((row & 15) << 3)) : row * LD + col;
  }
};

// One K step of a wave's FM x FN fragment grid.  The MFMA is issued with the B
// fragment as its first operand, so the 16x16 result is the C^T tile: lane l holds
// C[m = l & 15][n = 4 * (l >> 4) + r], r = 0..3 -- four consecutive columns of one row
// (vector stores in the epilogue, contiguous float4 split-K slabs).
template <int FM, int FN>
__device__ __forceinline__ void mfma_acc(f4v (&acc)[FM][FN], const bf16x8 (&af)[FM], const bf16x8 (&bfr)[FN]) {
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
}

// Shared epilogue: fp32 split-K slab store, or bf16 through LDS with bias /
// activation / pre-activation / act' / beta-accumulate / BN-statistics options.
// EPF > 1: plain / statistics bf16 epilogues read EPF staged rows from LDS before
// storing any (batched LDS latency; dense GEMMs only -- the conv loaders' registers leave
// no room, see docs/performance.md)
template <int BM, int BN, int WM, int WN, int EPI, int SMEM_SHORTS, int EPF = 1, int FM = BM / WM / 16,
          int FN = BN / WN / 16, bool QUAD = false, bool BIAS_IN_ACC = false>
__device__ __forceinline__ void gemm_epilogue(const CoreParams& P, f4v (&acc)[FM][FN], short* smem, int m0, int n0,
                                              int tm, int tid) {
  constexpr int NT = WM * WN * 64;
  using EL = EpiLayout<BN>;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  // accumulator layout (mfma_acc): acc[i][j][r] = C[frow(i)][fcol(j) + r].  Default: a wave owns
  // one (BM/WM) x (BN/WN) block, frow(i) = rbase + 16 i.  QUAD (the 8-phase 256 core): the tile
  // is four quadrants, each split over all waves -- a wave owns one (BM/2/WM) x (BN/2/WN) block
  // per quadrant, fragments i < FM/2 / j < FN/2 in the top / left quadrants.
  const int rbase = QUAD ? wm * (BM / 2 / WM) + (lane & 15) : wm * (BM / WM) + (lane & 15);
  const int cbase = QUAD ? wn * (BN / 2 / WN) + 4 * (lane >> 4) : wn * (BN / WN) + 4 * (lane >> 4);
  auto frow = [&](int i) { return QUAD ? rbase + (i / (FM / 2)) * (BM / 2) + (i % (FM / 2)) * 16 : rbase + i * 16; };
  auto fcol = [&](int j) { return QUAD ? cbase + (j / (FN / 2)) * (BN / 2) + (j % (FN / 2)) * 16 : cbase + j * 16; };
  if constexpr (EPI == EPI_F32_PARTIAL) {
    // N % 8 == 0 and ldc % 4 == 0 (slabs are [M][N]): a column group is whole or absent
    const BlkPos bp = blk_pos(P);
    float* Cp = reinterpret_cast<float*>(P.C) + (long)bp.split * P.split_stride;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int gm = m0 + frow(i), gn = n0 + fcol(j);
        if (gm < P.M && gn < P.N) *reinterpret_cast<f4v*>(Cp + (long)gm * P.ldc + gn) = acc[i][j];
      }
    // (an in-launch combine -- the last-arriving split summing all slabs behind an agent-scope
    // ticket -- measured 3-4x slower than the separate streaming reduce and was removed)
    return;
  } else {
    short* Cs = smem;
    if (!BIAS_IN_ACC && P.bias) {  // (BIAS_IN_ACC: the core started its accumulators at the bias)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int gn = n0 + fcol(j) + r;
          const float bv = gn < P.N ? P.bias[gn] : 0.f;
#pragma unroll
          for (int i = 0; i < FM; ++i) acc[i][j][r] += bv;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        s4v pk;
#pragma unroll
        for (int r = 0; r < 4; ++r) pk[r] = (short)f2bf(acc[i][j][r]);
        *reinterpret_cast<s4v*>(Cs + EL::idx(frow(i), fcol(j))) = pk;
      }
    __syncthreads();
    const bool fx = P.act != ACT_NONE || P.dact_src != nullptr || P.preact != nullptr;
    bf16_t* Cg = reinterpret_cast<bf16_t*>(P.C);
    float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, bzsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    (void)bsum;
    (void)bzsum;
    // Each thread owns one 8-column group (NT is a multiple of BN/8) and walks IT rows.
    // The global reads of the epilogue (old C for beta, BN input z and ReLU mask for
    // the BN-backward statistics) are issued PF rows at a time before any is used, so
    // a tile pays ceil(IT/PF) memory round trips instead of IT.
    constexpr int CH = BM * BN / 8;
    static_assert(CH % NT == 0, "epilogue chunks must divide the threads");
    constexpr int IT = CH / NT;
    constexpr bool Z2 = EPI == EPI_BF16_BNR2;
    constexpr bool BNS = EPI == EPI_BF16_BN || EPI == EPI_BF16_BNR || Z2, STS = EPI == EPI_BF16_ST;
    constexpr bool RSTAT = BNS || STS;
    float bz2sum[Z2 ? 8 : 1];
#pragma unroll
    for (int j = 0; j < (Z2 ? 8 : 1); ++j) bz2sum[j] = 0.f;
    constexpr bool RES = EPI != EPI_BF16_BN;  // res_src / res_mask compiled in
    // the calling core's LDS (SMEM_SHORTS bf16 slots) must hold the three statistics rows
    static_assert(!Z2 || 3 * (NT / (BN / 8)) * BN * 4 <= 2 * SMEM_SHORTS, "three statistics rows must fit the LDS");
    constexpr int PF = BNS ? (IT < 2 ? IT : 2) : (IT < EPF ? IT : EPF);
    // FIXCOL: NT is a multiple of BN / 8, so a thread keeps one 8-column group for every row it
    // walks (the statistics epilogues need that); otherwise (BN = 96 on 256 threads, plain
    // epilogues only) the column group follows the chunk index
    constexpr bool FIXCOL = NT % (BN / 8) == 0;
    static_assert(FIXCOL || (!RSTAT && EPI == EPI_BF16), "column groups must divide the threads");
    const int col0 = (tid % (BN / 8)) * 8;
    const bool has_beta = P.beta != 0.f;
#pragma unroll 1
    for (int it0 = 0; it0 < IT; it0 += PF) {
      s8v opre[PF], zpre[BNS ? PF : 1], zpre2[Z2 ? PF : 1], dsrc[RSTAT ? 1 : PF];
      uint32_t mk[PF];  // bits 0-7: BN ReLU mask (BN-backward statistics), bits 8-15: res_mask
      long orow[PF];
      bool okr[PF];
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        const int gm = m0 + (tid + (it0 + u) * NT) / (BN / 8);
        const int gn = n0 + (FIXCOL ? col0 : ((tid + (it0 + u) * NT) % (BN / 8)) * 8);
        okr[u] = gm < P.M && gn < P.N;
        orow[u] = okr[u] ? out_row(P, gm) : 0;
        const bf16_t* bsrc = (RES && P.res_src) ? P.res_src : Cg;
        opre[u] = (has_beta && okr[u] && beta_row_stored(P, orow[u]))
                      ? *reinterpret_cast<const s8v*>(bsrc + orow[u] * P.ldc + gn)
                      : zero8();
        mk[u] = 0xff00u;
        if constexpr (!RSTAT) {
          dsrc[u] = (P.dact_src && okr[u]) ? *reinterpret_cast<const s8v*>(P.dact_src + (long)gm * P.ld_aux + gn)
                                           : zero8();
        }
        if constexpr (RES) {
          if (has_beta && P.res_mask && okr[u]) mk[u] = (uint32_t)P.res_mask[orow[u] * (P.N / 8) + (gn >> 3)] << 8;
        }
        if constexpr (BNS) {
          zpre[u] = okr[u] ? *reinterpret_cast<const s8v*>(P.bnz + orow[u] * P.ldc + gn) : zero8();
          mk[u] |= (P.bnmask && okr[u]) ? (uint32_t)P.bnmask[orow[u] * (P.N / 8) + (gn >> 3)] : 0xffu;
        }
        if constexpr (Z2) zpre2[u] = okr[u] ? *reinterpret_cast<const s8v*>(P.bnz2 + orow[u] * P.ldc + gn) : zero8();
      }
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        if (!okr[u]) continue;
        const int row = (tid + (it0 + u) * NT) / (BN / 8);
        const int col = FIXCOL ? col0 : ((tid + (it0 + u) * NT) % (BN / 8)) * 8;
        const int gn = n0 + col;
        const int gm = m0 + row;
        s8v v = *reinterpret_cast<const s8v*>(Cs + EL::idx(row, col));
        bf16_t* dst = Cg + orow[u] * P.ldc + gn;
        if (fx) {
          if (P.preact) *reinterpret_cast<s8v*>(P.preact + (long)gm * P.ld_aux + gn) = v;
          if (P.dact_src) {
            const s8v src = RSTAT ? *reinterpret_cast<const s8v*>(P.dact_src + (long)gm * P.ld_aux + gn) : dsrc[RSTAT ? 0 : u];
            if (P.act == ACT_GELU) {
              gelu_grad_mul8(v, src);
            } else {
#pragma unroll
              for (int j = 0; j < 8; ++j)
                v[j] = (short)f2bf(bf2f((bf16_t)v[j]) * act_grad(P.act, bf2f((bf16_t)src[j])));
            }
          } else if (P.act == ACT_GELU) {
            gelu8(v);
          } else if (P.act != ACT_NONE) {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = (short)f2bf(act_fwd(P.act, bf2f((bf16_t)v[j])));
          }
        }
        if (has_beta) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float o = ((mk[u] >> (8 + j)) & 1u) ? bf2f((bf16_t)opre[u][j]) : 0.f;
            v[j] = (short)f2bf(bf2f((bf16_t)v[j]) + P.beta * o);
          }
        }
        if (!RSTAT && P.stats && (fx || has_beta)) *reinterpret_cast<s8v*>(Cs + EL::idx(row, col)) = v;
        *reinterpret_cast<s8v*>(dst) = v;
        if constexpr (STS) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float a = bf2f((bf16_t)v[j]);
            bsum[j] += a;
            bzsum[j] += a * a;
          }
        }
        if constexpr (BNS) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float g = ((mk[u] >> j) & 1u) ? bf2f((bf16_t)v[j]) : 0.f;
            bsum[j] += g;
            bzsum[j] += g * bf2f((bf16_t)zpre[u][j]);
            if constexpr (Z2) bz2sum[j] += g * bf2f((bf16_t)zpre2[u][j]);
          }
        }
      }
    }
    if constexpr (RSTAT) {
      // [sum | second moment] per column: registers -> LDS -> one thread per column
      constexpr int CG = BN / 8, PARTS = NT / CG;
      static_assert(NT % CG == 0, "column groups must divide the threads");
      const int cg = tid % CG, part = tid / CG;
      __syncthreads();  // Cs (aliases sred) fully consumed
      float* sred = reinterpret_cast<float*>(smem);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sred[part * BN + cg * 8 + j] = bsum[j];
        sred[(PARTS + part) * BN + cg * 8 + j] = bzsum[j];
        if constexpr (Z2) sred[(2 * PARTS + part) * BN + cg * 8 + j] = bz2sum[j];
      }
      __syncthreads();
      for (int c = tid; c < BN; c += NT) {
        if (n0 + c >= P.N) continue;
        float ts = 0.f, tq = 0.f, t2 = 0.f;
        for (int pp = 0; pp < PARTS; ++pp) {
          ts += sred[pp * BN + c];
          tq += sred[(PARTS + pp) * BN + c];
          if constexpr (Z2) t2 += sred[(2 * PARTS + pp) * BN + c];
        }
        // partial rows are per 128 GEMM rows (host-sized): a 256-row tile writes its sums
        // into the first of its two rows and zeros into the second (when it exists)
        constexpr int SR = BM >= 128 ? BM / 128 : 1;
        const bool zrow = SR == 2 && (long)(tm * 2 + 1) * 128 < P.M;
        float* st = P.stats + (long)tm * SR * 2 * P.N;
        st[n0 + c] = ts;
        st[P.N + n0 + c] = tq;
        if (zrow) {
          st[2 * P.N + n0 + c] = 0.f;
          st[3 * P.N + n0 + c] = 0.f;
        }
        if constexpr (Z2) {
          float* st2 = P.stats2 + (long)tm * SR * 2 * P.N;
          st2[n0 + c] = ts;
          st2[P.N + n0 + c] = t2;
          if (zrow) {
            st2[2 * P.N + n0 + c] = 0.f;
            st2[3 * P.N + n0 + c] = 0.f;
          }
        }
      }
    } else if (FIXCOL && NT % BN == 0 && P.stats) {  // (host: never set for other tiles)
      // per-column sum / sum of squares of the stored bf16 values of this tile
      constexpr int TPC = NT / BN;
      const int col = tid % BN, part = tid / BN;
      float s = 0.f, q = 0.f;
      int rows = P.M - m0;
      if (rows > BM) rows = BM;
      __syncthreads();
      for (int r = part; r < rows; r += TPC) {
        const float v = bf2f((bf16_t)Cs[EL::idx(r, col)]);
        s += v;
        q += v * v;
      }
      __syncthreads();
      float* sred = reinterpret_cast<float*>(smem);
      sred[part * BN + col] = s;
      sred[(TPC + part) * BN + col] = q;
      __syncthreads();
      if (part == 0 && n0 + col < P.N) {
        float ts = 0.f, tq = 0.f;
#pragma unroll
        for (int pp = 0; pp < TPC; ++pp) {
          ts += sred[pp * BN + col];
          tq += sred[(TPC + pp) * BN + col];
        }
        constexpr int SR = BM >= 128 ? BM / 128 : 1;
        float* st = P.stats + (long)tm * SR * 2 * P.N;
        st[n0 + col] = ts;
        st[P.N + n0 + col] = tq;
        if (SR == 2 && (long)(tm * 2 + 1) * 128 < P.M) {
          st[2 * P.N + n0 + col] = 0.f;
          st[3 * P.N + n0 + col] = 0.f;
        }
      }
    }
  }
}

// ------------------------------------------------------------------ core --
template <int BM, int BN, int WM, int WN, template <int, int, int> class LAT, template <int, int, int> class LBT,
          int EPI, int NSTAGE = 2>
__device__ __forceinline__ void mfma_gemm_body(const CoreParams& P) {
  constexpr int NT = WM * WN * 64;
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;
  constexpr bool A_KC = LAT<BM, 1, NT>::KC, B_KC = LBT<BN, 1, NT>::KC;
  using GA = TileGeom<BM, A_KC>;
  using GB = TileGeom<BN, B_KC>;
  constexpr int STAGE = GA::ELEMS + GB::ELEMS;
  constexpr int EPI_LD = EpiLayout<BN>::LD;
  constexpr int SMEM = (NSTAGE * STAGE > BM * EPI_LD ? NSTAGE * STAGE : BM * EPI_LD);
  constexpr int CPA = GA::CHUNKS / NT, CPB = GB::CHUNKS / NT;
  using LA = LAT<BM, CPA, NT>;
  using LB = LBT<BN, CPB, NT>;
  static_assert(GA::CHUNKS % NT == 0 && GB::CHUNKS % NT == 0, "tile chunks must divide threads");
  __shared__ __attribute__((aligned(16))) short smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_m = (P.M + BM - 1) / BM, tiles_n = (P.N + BN - 1) / BN;
  const BlkPos bp = blk_pos(P);
  const int tm = bp.tile / tiles_n, tn = bp.tile % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = bp.split * P.k_per_split;
  int kend = kbeg + P.k_per_split;
  if (kend > P.K) kend = P.K;
  const int nk = (kend - kbeg + BK - 1) / BK;

  const LA la(P, true, m0, tid);
  const LB lb(P, false, n0, tid);
  s8v ra[CPA], rb[CPB];
  int arow[CPA], acol[CPA], brow[CPB], bcol[CPB];
#pragma unroll
  for (int i = 0; i < CPA; ++i) chunk_coords<BM, A_KC>(tid + i * NT, arow[i], acol[i]);
#pragma unroll
  for (int i = 0; i < CPB; ++i) chunk_coords<BN, B_KC>(tid + i * NT, brow[i], bcol[i]);

  f4v acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < CPA; ++i) ra[i] = la.load(i, k0);
#pragma unroll
    for (int i = 0; i < CPB; ++i) rb[i] = lb.load(i, k0);
  };
  auto lstore = [&](short* base) {
#pragma unroll
    for (int i = 0; i < CPA; ++i) *reinterpret_cast<s8v*>(base + arow[i] * GA::LD + acol[i]) = ra[i];
#pragma unroll
    for (int i = 0; i < CPB; ++i) *reinterpret_cast<s8v*>(base + GA::ELEMS + brow[i] * GB::LD + bcol[i]) = rb[i];
  };

  auto compute = [&](const short* As) {
    const short* Bs = As + GA::ELEMS;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = read_frag<BM, A_KC>(As, wm * (BM / WM) + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = read_frag<BN, B_KC>(Bs, wn * (BN / WN) + j * 16, kk, lane);
      mfma_acc<FM, FN>(acc, af, bfr);
    }
  };
  if constexpr (NSTAGE == 1) {
    for (int t = 0; t < nk; ++t) {
      gload(kbeg + t * BK);
      if (t) __syncthreads();
      lstore(smem);
      __syncthreads();
      compute(smem);
    }
    __syncthreads();
  } else {
    if (nk > 0) {
      gload(kbeg);
      lstore(smem);
    }
    __syncthreads();
    int cur = 0;
    for (int t = 0; t < nk; ++t) {
      const bool more = (t + 1) < nk;
      if (more) gload(kbeg + (t + 1) * BK);
      compute(smem + cur * STAGE);
      if (more) lstore(smem + (cur ^ 1) * STAGE);
      __syncthreads();
      cur ^= 1;
    }
  }

  gemm_epilogue<BM, BN, WM, WN, EPI, SMEM>(P, acc, smem, m0, n0, tm, tid);
}

// ======================================================= LDS-DMA (glds) core --
// Operand tiles are filled by global_load_lds_dwordx4 (16 B per lane straight
// into LDS, no VGPR round trip, no ds_write pass).  The LDS image of a wave
// instruction is lane-linear, so tiles are UNPADDED and bank conflicts are
// removed by an XOR swizzle applied on the SOURCE side (each lane fetches the
// logical chunk that belongs at its linear slot) and undone by the readers:
//   K-contiguous tile [rows][64]  (8 x 16-B chunks per 128-B row):
//       phys = logical ^ (row & 7)       -> ds_read_b128 fragment reads conflict-free
//   N-contiguous tile [64 k][R]   (R/8 chunks per row), transposed reads:
//       R = 128: phys = logical ^ 2*((k&3) | ((k>>3)&1)<<2)
//       R =  64: phys = logical ^ 2*(((k>>1)&1) | ((k>>3)&1)<<1)
//     -> the 8 k-rows one ds_read_b64_tr_b16 half-wave touches land in 8
//        distinct 32-B bank slots.
// Out-of-range K chunks read a 16-B zero page (rows/cols beyond M/N are clamped:
// they only feed outputs that are never stored).  One LDS stage, two barriers
// per K step; several blocks per CU hide the DMA latency.

static __device__ __attribute__((aligned(16))) bf16_t ca_zero16[8];

typedef __attribute__((address_space(3))) void lds_void;

// Branch-free choice between a chunk's source address and the zero page.  Written as a
// mask on the address bits: a plain `ok ? a : zero` lets the compiler sink the address
// arithmetic into an exec-masked branch per chunk (measured: 2 branches + ~20 SALU per
// chunk in the DMA issue sequence of the gather loaders).
__device__ __forceinline__ const bf16_t* sel_src(bool ok, const bf16_t* a) {
  const uint64_t m = 0 - (uint64_t)ok;
  return reinterpret_cast<const bf16_t*>((reinterpret_cast<uint64_t>(a) & m) |
                                         (reinterpret_cast<uint64_t>(ca_zero16) & ~m));
}

// Buffer-mode loaders (static constexpr bool BUF = true): a block-uniform base `sbase`, a
// byte range `nrec`, and per chunk a 32-bit byte offset from off(i, k0).  The DMA is a
// buffer_load_dwordx4 ... lds through a resource built once per operand; a lane whose
// offset is >= nrec (loaders return nrec itself for padding taps, K tails and rows past the
// operand) gets ZEROS in its LDS slot from the hardware range check -- probed on gfx950,
// scripts/debug/buffer_lds_oob_probe.hip -- so there is no zero page, no 64-bit address
// arithmetic and no select on 64-bit pointers in the issue sequence.
// (BUF_CAP / buf_span: top of this file)

template <class L, class = void>
struct loader_buf {
  static constexpr bool value = false;
};
template <class L>
struct loader_buf<L, decltype((void)L::BUF)> {
  static constexpr bool value = L::BUF;
};

template <class L>
__device__ __forceinline__ auto loader_rsrc(const L& l) {
  if constexpr (loader_buf<L>::value)
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(l.sbase), (short)0, (int)l.nrec, 0x00020000);
  else
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(ca_zero16), (short)0, 0, 0x00020000);
}

// one 16-B chunk per lane into the lane-linear LDS slot at dst (buffer- or pointer-mode loader)
#define CA_DMA_CHUNK(L, l, r, i, k0, dst)                                                           \
  do {                                                                                              \
    if constexpr (loader_buf<L>::value)                                                             \
      __builtin_amdgcn_raw_ptr_buffer_load_lds((r), (lds_void*)(dst), 16, (l).off((i), (k0)), 0, 0, 0); \
    else                                                                                            \
      __builtin_amdgcn_global_load_lds((const void*)(l).src((i), (k0)), (lds_void*)(dst), 16, 0, 0);  \
  } while (0)

template <int R>
__device__ __forceinline__ int nc_swz(int k) {
  if constexpr (R >= 128) return 2 * ((k & 3) | (((k >> 3) & 1) << 2));
  else return 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1));
}

template <int R, bool KC>
__device__ __forceinline__ bf16x8 read_frag_sw(const short* lds, int r0, int k0, int lane) {
  if constexpr (KC) {
    const int row = r0 + (lane & 15);
    const int pc = ((k0 >> 3) + (lane >> 4)) ^ (row & 7);
    s8v v = *reinterpret_cast<const s8v*>(lds + row * BK + pc * 8);
    return __builtin_bit_cast(bf16x8, v);
  } else {
    const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
    const int k = k0 + 8 * g + q;
    const int lc = (r0 >> 3) + (p >> 1);
    const int sub = 4 * (p & 1);
    const short* b0 = lds + k * R + ((lc ^ nc_swz<R>(k)) << 3) + sub;
    const short* b1 = lds + (k + 4) * R + ((lc ^ nc_swz<R>(k + 4)) << 3) + sub;
    s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(b0));
    s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(b1));
    s8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// Loader address rule (all glds loaders): everything that varies per lane is folded into
// per-chunk pointers in the constructor, so a K tile adds only a wave-uniform offset
// (computed on the scalar unit) -- no per-tile integer multiplies, which are quarter-rate
// on the VALU.  Measured before this rule (counter pass, ResNet-50): 140-210 VALU per K tile
// per wave in the convolution loaders against 16-32 MFMAs, i.e. the SIMD's issue slots, not
// the matrix pipe, bounded the implicit-GEMM kernels.

// Dense K-contiguous operand for the glds core: X[r][k] at p[r*ld + k].
// Chunk i of thread tid covers tile row (tid>>3) + i*(NT/8) and the swizzled
// column slot (tid&7) ^ (row&7) -- the XOR term is the same for every i.
template <int R, int CPT, int NT>
struct GDenseKC {
  static constexpr bool KC = true, BUF = true;
  const bf16_t* sbase;  // &X[r0][0] (block-uniform)
  uint32_t nrec;        // bytes from sbase to the end of the operand's last row
  uint32_t roff;        // (row * ld + col) * 2 of chunk 0
  uint32_t ldb2;        // ld * 2
  int col, K;
  __device__ GDenseKC(const CoreParams& P, bool isA, int r0, int tid) {
    const bf16_t* p = isA ? P.A : P.B;
    const long ld = isA ? P.lda : P.ldb;
    const int rows = isA ? P.M : P.N;
    K = P.K;
    const int row = tid >> 3;
    col = ((tid & 7) ^ (row & 7)) << 3;
    sbase = p + (long)r0 * ld;
    // rows at or past `rows` start at byte (rows - r0) * ld * 2 >= nrec: read as zeros
    nrec = buf_span((long)(rows - r0) * ld * 2);
    ldb2 = (uint32_t)(ld * 2);
    roff = (uint32_t)((row * ld + col) * 2);
  }
  __device__ __forceinline__ uint32_t off(int i, int k0) const {
    const uint32_t o = roff + (uint32_t)(i * (NT / 8)) * ldb2 + (uint32_t)k0 * 2u;
    return (k0 + col < K) ? o : nrec;
  }
};

// Dense output-dim-contiguous operand for the glds core: X[r][k] at p[k*ld + r].
// Chunk i covers k-row (tid / (R/8)) + i * (NT*8/R); its swizzle term is i-invariant.
template <int R, int CPT, int NT>
struct GDenseNC {
  static constexpr bool KC = false, BUF = true;
  static constexpr int KSTEP = NT * 8 / R;
  const bf16_t* sbase;  // &X[kbeg][0]: the block's first reduction row (split-K start)
  uint32_t nrec;
  uint32_t coff;  // (krow0 * ld + n) * 2
  uint32_t ldb2;
  int krow0, kbeg, K;
  __device__ GDenseNC(const CoreParams& P, bool isA, int r0, int tid) {
    const bf16_t* p = isA ? P.A : P.B;
    const long ld = isA ? P.lda : P.ldb;
    const int rlimit = isA ? P.M : P.N;
    K = P.K;
    constexpr int CPR = R / 8;  // chunks per k-row
    const int k = tid / CPR, pc = tid % CPR;
    int n = r0 + ((pc ^ nc_swz<R>(k)) << 3);
    // launchers guarantee rlimit % 8 == 0 and rlimit >= 8 (N < 8 is refused host-side); the
    // clamp keeps a fully out-of-range column chunk on the last real one
    if (n > rlimit - 8) n = rlimit - 8 > 0 ? rlimit - 8 : 0;
    krow0 = k;
    kbeg = blk_split(P) * P.k_per_split;
    sbase = p + (long)kbeg * ld;
    nrec = buf_span(((long)(K - kbeg - 1) * ld + rlimit) * 2);
    ldb2 = (uint32_t)(ld * 2);
    coff = (uint32_t)((k * ld + n) * 2);
  }
  __device__ __forceinline__ uint32_t off(int i, int k0) const {
    const uint32_t o = coff + (uint32_t)(k0 - kbeg + i * KSTEP) * ldb2;
    return (k0 + krow0 + i * KSTEP < K) ? o : nrec;
  }
};

// Loaders that keep per-chunk state walked forward one K tile at a time define advance();
// the cores call it after issuing each tile of that operand (tiles are issued in order).
template <class L, class = void>
struct loader_stateful {
  static constexpr bool value = false;
};
template <class L>
struct loader_stateful<L, decltype((void)&L::advance)> {
  static constexpr bool value = true;
};

template <int BM, int BN, int WM, int WN, template <int, int, int> class LAT, template <int, int, int> class LBT,
          int EPI, int NSTAGE = 1, int EPF = 1>
__device__ __forceinline__ void mfma_gemm_glds(const CoreParams& P) {
  // Measured on MI355X (bench/conv_shapes.py, bench/gemm_core_ab.py): NSTAGE 1 at
  // 4 blocks/CU beats NSTAGE 2 at 2 blocks/CU by 10-15% on every ResNet/BERT shape.
  // NSTAGE 1: load -> wait -> barrier -> MFMA -> barrier; latency hidden by ~4
  //           co-resident blocks (34 KB LDS each).
  // NSTAGE 2: the DMA of K tile t+1 is in flight while tile t is multiplied; a
  //           counted s_waitcnt vmcnt(loads per tile) retires exactly tile t and
  //           RAW s_barriers (not __syncthreads, whose fence would drain the
  //           in-flight DMA with vmcnt(0)) order the LDS image.
  constexpr int NT = WM * WN * 64;
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;
  constexpr int A_ELEMS = BM * BK, B_ELEMS = BN * BK;
  constexpr int STAGE = A_ELEMS + B_ELEMS;
  constexpr int EPI_LD = EpiLayout<BN>::LD;
  constexpr int SMEM = (NSTAGE * STAGE > BM * EPI_LD ? NSTAGE * STAGE : BM * EPI_LD);
  constexpr int CPA = A_ELEMS / 8 / NT, CPB = B_ELEMS / 8 / NT;
  using LA = LAT<BM, CPA, NT>;
  using LB = LBT<BN, CPB, NT>;
  constexpr bool A_KC = LA::KC, B_KC = LB::KC;
  static_assert(A_ELEMS % (8 * NT) == 0 && B_ELEMS % (8 * NT) == 0, "tile chunks must divide threads");
  static_assert(CPA + CPB < 64, "vmcnt range");
  __shared__ __attribute__((aligned(16))) short smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_m = (P.M + BM - 1) / BM, tiles_n = (P.N + BN - 1) / BN;
  const BlkPos bp = blk_pos(P);
  const int tm = bp.tile / tiles_n, tn = bp.tile % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = bp.split * P.k_per_split;
  int kend = kbeg + P.k_per_split;
  if (kend > P.K) kend = P.K;
  const int nk = (kend - kbeg + BK - 1) / BK;

  LA la(P, true, m0, tid);
  LB lb(P, false, n0, tid);

  // dense-layer bias: the accumulators START at the bias (loaded before the K loop, its latency
  // under the first DMA; no registers beyond the accumulators) and the epilogue skips its own
  // bias add -- which waited one memory round trip per tile (BERT FFN1 forward: +11 us per call)
  f4v acc[FM][FN];
  constexpr bool BIAS0 = EPI == EPI_BF16;
  // (addresses clamped instead of branched so the 16 loads go out back to back.  Issuing them
  // behind the first K tile's DMA instead -- first tile peeled -- measured no better)
  auto init_acc = [&]() {
    if (BIAS0 && P.bias) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        f4v b;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int gn = n0 + wn * (BN / WN) + 4 * (lane >> 4) + j * 16 + r;
          const float v = P.bias[gn < P.N ? gn : P.N - 1];
          b[r] = gn < P.N ? v : 0.f;
        }
#pragma unroll
        for (int i = 0; i < FM; ++i) acc[i][j] = b;
      }
    } else {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
    }
  };

  const auto ra = loader_rsrc(la);
  const auto rb = loader_rsrc(lb);
  auto issue = [&](int t, short* base) {
    const int k0 = kbeg + t * BK;
#pragma unroll
    for (int i = 0; i < CPA; ++i) CA_DMA_CHUNK(LA, la, ra, i, k0, base + (i * NT + wave * 64) * 8);
#pragma unroll
    for (int i = 0; i < CPB; ++i) CA_DMA_CHUNK(LB, lb, rb, i, k0, base + A_ELEMS + (i * NT + wave * 64) * 8);
    if constexpr (loader_stateful<LA>::value) la.advance();
    if constexpr (loader_stateful<LB>::value) lb.advance();
  };
  auto compute = [&](const short* As) {
    const short* Bs = As + A_ELEMS;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = read_frag_sw<BM, A_KC>(As, wm * (BM / WM) + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = read_frag_sw<BN, B_KC>(Bs, wn * (BN / WN) + j * 16, kk, lane);
      mfma_acc<FM, FN>(acc, af, bfr);
    }
  };

  init_acc();
  if constexpr (NSTAGE == 1) {
    for (int t = 0; t < nk; ++t) {
      issue(t, smem);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      compute(smem);
      __syncthreads();
    }
  } else {
    if (nk > 0) issue(0, smem);
    for (int t = 0; t < nk; ++t) {
      if (t + 1 < nk) {
        issue(t + 1, smem + ((t + 1) & 1) * STAGE);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(CPA + CPB) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      compute(smem + (t & 1) * STAGE);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }
  gemm_epilogue<BM, BN, WM, WN, EPI, SMEM, EPF, FM, FN, false, BIAS0>(P, acc, smem, m0, n0, tm, tid);
}

}  // namespace ca
