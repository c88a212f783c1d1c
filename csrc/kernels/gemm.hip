// Dense bf16 MFMA GEMMs for 1x1 NHWC convolutions and dense layers (K1).
//
//   layout 0 "NT": C[M,N] = A[M,K] * B[N,K]^T   forward      Y  = X  W^T
//   layout 1 "NN": C[M,N] = A[M,K] * B[K,N]     input grad   dX = dY W
//   layout 2 "TN": C[M,N] = A[K,M]^T * B[K,N]   weight grad  dW = dY^T X  (split-K)
//
// All three read the tensors exactly as they lie in memory; the core
// (csrc/include/ca_mfma_core.h) stages K-contiguous tiles for ds_read_b128
// and M/N-contiguous tiles for the gfx950 transposed read ds_read_b64_tr_b16.
// Split-K writes fp32 slabs reduced deterministically by splitk_reduce_kernel.
#include <stdlib.h>
#include <string.h>

#include "ca_gemm256p8.h"
#include "ca_gemm_xa.h"

// Experiment-only cores -- the 8-wave glds8 variant, the 256 x 256 ring core, stream-K and the
// 256 x 128 variant -- each measured slower than the default dispatch (docs/performance.md) and
// kept for A/B runs: compiled only with CLOUD_AMD_BUILD_EXPERIMENTAL=1 (-DCA_EXPERIMENTAL=1).
#ifndef CA_EXPERIMENTAL
#define CA_EXPERIMENTAL 0
#endif

namespace {
using namespace ca;

template <int BM, int BN, template <int, int, int> class LA, template <int, int, int> class LB, int EPI, int NS>
__global__ void __launch_bounds__(256) dense_gemm_kernel(CoreParams P) {
  mfma_gemm_body<BM, BN, 2, 2, LA, LB, EPI, NS>(P);
}

template <int BM, int BN, template <int, int, int> class LA, template <int, int, int> class LB, int EPI>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) dense_gemm_glds_kernel(CoreParams P) {
  mfma_gemm_glds<BM, BN, 2, 2, LA, LB, EPI>(P);
}

// same, with the statistics epilogue reading 4 staged rows ahead of their stores
template <int BM, int BN, template <int, int, int> class LA, template <int, int, int> class LB, int EPI>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) dense_gemm_glds_pf_kernel(CoreParams P) {
  mfma_gemm_glds<BM, BN, 2, 2, LA, LB, EPI, 1, 4>(P);
}

// Forward GEMMs with the BN-statistics epilogue (ResNet 1x1 convs) use the batched
// epilogue: fwd1x1 3.2M x 256 x 64 501 -> 463 us, 802K x 512 x 128 315 -> 300 us, ResNet-50
// b1024 +0.9 %.  Plain bias/activation epilogues (BERT) measured 0.8 % slower with it, so
// they keep one row per trip.  CLOUD_AMD_EPI_PF=0 turns it off (A/B runs).
bool epi_pf() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CLOUD_AMD_EPI_PF");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v != 0;
}

// 256 x 96 tiles for forward GEMMs whose 128 x 128 grid ends in a partial round while the
// 256 x 96 grid fills whole rounds (BERT's QKV projection, M = 8192, N = 2304: 1,152 tiles =
// 4.5 rounds vs 768 = 3; 41.9 -> 36.8 us, profiles/r5_s9/r5s9_gb.log)
template <int EPI>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) dense_gemm_256x96_kernel(CoreParams P) {
  mfma_gemm_glds<256, 96, 2, 2, GDenseKC, GDenseKC, EPI>(P);
}

#if CA_EXPERIMENTAL
// 8 waves (2 x 4, wave tile 64 x BN/4) with a double-buffered LDS-DMA pipeline:
// same 16 waves/CU occupancy as the 4-wave single-stage kernel, but the next K
// tile's DMA overlaps this tile's MFMAs (CLOUD_AMD_GEMM_CORE=glds8).
template <int BM, int BN, template <int, int, int> class LA, template <int, int, int> class LB, int EPI>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) dense_gemm_glds8_kernel(CoreParams P) {
  mfma_gemm_glds<BM, BN, 2, 4, LA, LB, EPI, 2>(P);
}
#endif  // CA_EXPERIMENTAL

#if CA_EXPERIMENTAL
// The 256 x 256 ring core (csrc/include/ca_gemm256.h) for large GEMMs: one 512-thread
// workgroup per CU.  K-contiguous operands use the 32-deep KC32 loader, N-contiguous ones
// the same GDenseNC loader as the 128 cores.
template <template <int, int, int> class LA, template <int, int, int> class LB, int EPI>
__global__ void __launch_bounds__(512) dense_gemm_256_kernel(CoreParams P) {
  mfma_gemm_256<LA, LB, EPI>(P);
}
#endif  // CA_EXPERIMENTAL

// The 256 x 256 x 64 core with two staggered wave groups and two phases per K tile
// (csrc/include/ca_gemm256p8.h).
template <template <int, int, int> class LA, template <int, int, int> class LB, int EPI>
__global__ void __launch_bounds__(512) dense_gemm_256p8_kernel(CoreParams P) {
  mfma_gemm_256p8<LA, LB, EPI, 2>(P);
}

#if CA_EXPERIMENTAL
// Stream-K form of the same core (ca_gemm256p8.h mfma_gemm_256p8_sk): one workgroup per CU,
// each an equal range of the (tile, K iteration) space.
template <template <int, int, int> class LA, template <int, int, int> class LB, int EPI>
__global__ void __launch_bounds__(512) dense_gemm_256p8_sk_kernel(CoreParams P, SkParams S) {
  mfma_gemm_256p8_sk<LA, LB, EPI>(P, S);
}

// Its 256 x 128 single-phase, three-buffer variant (same header).
template <template <int, int, int> class LA, template <int, int, int> class LB, int EPI>
__global__ void __launch_bounds__(512) dense_gemm_256x128_kernel(CoreParams P) {
  mfma_gemm_256x128<LA, LB, EPI>(P);
}
#endif  // CA_EXPERIMENTAL

// CLOUD_AMD_GEMM_CORE selects the core (A/B comparisons; ca_gemm_set_core overrides it):
// 0 "reg" = register-staged, 1 "glds" = glds single stage (4 waves) only, 2 "glds8" = glds
// double-buffered (8 waves), 3 "glds_ring" = glds plus the 256 x 256 ring core (ca_gemm256.h)
// for large GEMMs, 4 "v256" = the ring core for every GEMM with M, N >= 256 (tests),
// 5 (default) = glds plus the 256 x 256 two-phase core (ca_gemm256p8.h) for large GEMMs
// (use_256 below; 8192^3: ring 1,172-1,183 -> 1,245-1,260 TF/s, split-K / TN weight-gradient
// layout 1,042 -> 1,142), 6 "vp8" = the two-phase core for every GEMM with M, N >= 256 (tests).
int g_core_kind = -1;
int core_kind() {
  if (g_core_kind < 0) {
    const char* e = getenv("CLOUD_AMD_GEMM_CORE");
    g_core_kind = !e ? 5
                     : (e[0] == 'r' ? 0
                        : strcmp(e, "glds8") == 0     ? 2
                        : strcmp(e, "glds") == 0      ? 1
                        : strcmp(e, "glds_ring") == 0 ? 3
                        : strcmp(e, "v256") == 0      ? 4
                        : strcmp(e, "vp8") == 0       ? 6
                                                      : 5);
  }
#if !CA_EXPERIMENTAL
  if (g_core_kind >= 2 && g_core_kind <= 4) g_core_kind = 5;  // not built: the default dispatch
#endif
  return g_core_kind;
}
bool core_p8() { return core_kind() == 5 || core_kind() == 6; }
bool use_glds() { return core_kind() != 0; }

// Persistent resident-weight core (csrc/include/ca_gemm_prw.h) for the small-K forward 1x1
// convolutions with the BN-statistics epilogue.
template <int BN, int KT, int NS, bool STATS>
__global__ void __launch_bounds__(512) prw_gemm_kernel(CoreParams P) {
  prw_gemm_body<BN, KT, NS, STATS>(P);
}

// CLOUD_AMD_GEMM_PRW=0 keeps these GEMMs on the data-parallel 128 core (A/B runs)
bool prw_enabled() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CLOUD_AMD_GEMM_PRW");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v != 0;
}

int cu_count() {
  static int n = -1;
  if (n < 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    n = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess &&
         prop.multiProcessorCount > 0)
            ? prop.multiProcessorCount
            : 256;
  }
  return n;
}

// (N, K) -> instantiation id; 0 = not covered.  The whole [N][K] weight stays in LDS.
// Only N = 256, K = 64 (ResNet layer-1 conv3 and projection shortcut) is taken: measured on
// MI355X at M = 3.2M (bench/smallk_gemm.py, profiles/r3_s12, r3_s14), with statistics,
// persistent vs tiled 128 core:
//   N 256, K  64: 413-420 vs 492 us   (the tile's 128 x 256 output per 16 KB of A is where
//                                     overlapping the next tile's loads with the stores pays)
//   N  64, K 256: 403-418 vs 377 us   (ring depth 4 and 6)
//   N  64, K  64: 168 vs 155 us       (ring depth 3 and 8)
//   N 128, K 256: 468-492 vs 468 us
// so the other shapes stay on the tiled core, whose 4 co-resident blocks per CU already keep
// enough loads in flight for their read-heavy tiles.
// Column-chunked kinds (ca_gemm_prw.h "Column chunks"): ResNet's conv3 expansions, forward
// with statistics only -- N = 512 / K = 128 (stage 2, 4 chunks of 128) and N = 1024 / K = 256
// (stage 3, 8 of 128).  Measured at b1024 with statistics (bench/smallk_gemm.py, profiles/r6_s7,
// r6_s8): stage 2 334.6 -> 274-290 us, stage 3 218.6 -> 209-211 us; not taken: stage 4
// (N = 2048 / K = 512, 32 chunks of 64: 143.5 -> 270.6 us), ring depth 5 at stage 2 (no change),
// 16 chunks of 64 at stage 3 (296 us), and the chunks of a range spread over the XCDs instead
// of sharing one (211.8 vs 209.1 us: the A re-reads are not the bound -- the per-tile epilogue
// turnaround of one 8-wave workgroup per CU is).  CLOUD_AMD_GEMM_PRWN=0 keeps them on the tiled
// cores (A/B runs).
bool prwn_enabled() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CLOUD_AMD_GEMM_PRWN");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v != 0;
}

int prw_kind(int M, int N, int K, long lda, long ldb, long ldc, bool stats) {
  if (!prw_enabled() || lda != K || ldb != K || ldc != N || M < 128) return 0;
  if ((long)M * K * 2 >= (long)BUF_CAP || (long)M * N * 2 >= (long)BUF_CAP) return 0;
  if (N == 256 && K == 64) return 2;
  if (!stats || !prwn_enabled() || cu_count() % 256 != 0) return 0;
  if (N == 512 && K == 128) return 3;
  if (N == 1024 && K == 256) return 4;
  return 0;
}

// (BN, KT, NS, column chunks) of each kind
struct PrwCfg {
  int bn, kt, ns, chunks;
};
PrwCfg prw_cfg(int kind) {
  switch (kind) {
    case 2: return {256, 64, 3, 1};
    case 3: return {128, 128, 3, 4};
    case 4: return {128, 256, 3, 8};
    default: return {0, 0, 0, 0};
  }
}

template <int BN, int KT, int NS>
int prw_grid_for(int M, int chunks) {
  constexpr int bytes = PrwGeom<BN, KT, NS>::BYTES;
  static_assert(bytes <= 160 * 1024, "LDS");
  int per_cu = (160 * 1024) / bytes;
  if (per_cu > 4) per_cu = 4;
  const int tiles = (M + 127) / 128;
  if (chunks > 1) {
    // a multiple of 8 * chunks (the chunks of a range on one XCD), at most one range per tile
    const int unit = 8 * chunks;
    int ranges = (cu_count() * per_cu / unit) * 8;
    if (ranges > tiles) ranges = tiles / 8 * 8;
    return ranges < 8 ? 0 : ranges * chunks;
  }
  const int g = cu_count() * per_cu;
  return g < tiles ? g : tiles;
}

int prw_grid(int kind, int M) {
  switch (kind) {
    case 2: return prw_grid_for<256, 64, 3>(M, 1);
    case 3: return prw_grid_for<128, 128, 3>(M, 4);
    case 4: return prw_grid_for<128, 256, 3>(M, 8);
    default: return 0;
  }
}

// rows of the statistics partials: one per workgroup, or one per range with column chunks
int prw_stat_rows(int kind, int M) {
  const int g = prw_grid(kind, M);
  const int ch = prw_cfg(kind).chunks;
  return ch > 1 ? g / ch : g;
}

int prw_launch(int kind, const CoreParams& p0, hipStream_t s) {
  const int g = prw_grid(kind, p0.M);
  if (g <= 0) return -2;
  CoreParams p = p0;
  p.prw_chunks = prw_cfg(kind).chunks;
  const bool st = p.stats != nullptr;
#define CA_PRW(BN_, KT_, NS_)                                                             \
  do {                                                                                    \
    if (st) prw_gemm_kernel<BN_, KT_, NS_, true><<<g, 512, 0, s>>>(p);                    \
    else prw_gemm_kernel<BN_, KT_, NS_, false><<<g, 512, 0, s>>>(p);                      \
  } while (0)
  switch (kind) {
    case 2: CA_PRW(256, 64, 3); break;
    case 3: CA_PRW(128, 128, 3); break;
    case 4: CA_PRW(128, 256, 3); break;
    default: return -2;
  }
#undef CA_PRW
  CA_LAUNCH_CHECK();
  return 0;
}

template <bool OUT_BF16>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ ws, int S, long MN,
                                                           void* __restrict__ out, float beta, int CB) {
  // block = CB float4-columns x (256/CB) slab-lanes; LDS tree over the slab-lanes.
  __shared__ f4v red[256];
  const long n4 = MN / 4;
  const int SL = 256 / CB;
  const int col = threadIdx.x % CB, sl = threadIdx.x / CB;
  const long v = (long)blockIdx.x * CB + col;
  f4v acc = {0.f, 0.f, 0.f, 0.f};
  if (v < n4) {
#pragma unroll 4
    for (int s = sl; s < S; s += SL) acc += *reinterpret_cast<const f4v*>(ws + (long)s * MN + v * 4);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = SL / 2; w > 0; w >>= 1) {
    if (sl < w) red[threadIdx.x] += red[threadIdx.x + w * CB];
    __syncthreads();
  }
  if (sl != 0 || v >= n4) return;
  acc = red[col];
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

// Split-K reduce of a LARGE output (>= 64 x 512 float4 columns): one float4 column per thread,
// every slab's load issued back to back (S loads of 16 B in flight per thread instead of the
// tree kernel's 1-2), summed in slab order 0..S-1.  The tree kernel above reached ~2.5 TB/s on
// BERT's weight gradients (6 slabs of 2304 x 768: 1-2 dependent loads per thread, two LDS
// barriers per 1 KB of output); this form streams.  The small-output case keeps the tree
// (slab-lanes give it the parallelism its few columns lack).
template <bool OUT_BF16>
__global__ void __launch_bounds__(256) splitk_reduce_cols_kernel(const float* __restrict__ ws, int S, long MN,
                                                                void* __restrict__ out, float beta) {
  const long n4 = MN / 4;
  const long v = (long)blockIdx.x * 256 + threadIdx.x;
  if (v >= n4) return;
  const f4v* p = reinterpret_cast<const f4v*>(ws) + v;
  f4v acc = p[0];
  int s = 1;
  for (; s + 4 <= S; s += 4) {
    const f4v a = p[(long)s * n4], b = p[(long)(s + 1) * n4], c = p[(long)(s + 2) * n4], d = p[(long)(s + 3) * n4];
    acc += a;
    acc += b;
    acc += c;
    acc += d;
  }
  for (; s < S; ++s) acc += p[(long)s * n4];
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

// Split-K reduce for a skinny dense layer (Keras Flatten -> Dense: small batch, long K):
// out[m][n] = act(sum_s ws[s][m][n] + bias[n]) in bf16 -- the fp32 sum, bias add, activation
// and cast of the layer in one pass (no fp32 output tensor, no elementwise kernels).
__global__ void __launch_bounds__(256) splitk_bias_act_kernel(const float* __restrict__ ws, int S, long M, int N,
                                                              const float* __restrict__ bias, int act,
                                                              bf16_t* __restrict__ out) {
  const long n4 = M * N / 4;
  for (long v = (long)blockIdx.x * 256 + threadIdx.x; v < n4; v += (long)gridDim.x * 256) {
    f4v acc = {0.f, 0.f, 0.f, 0.f};
    for (int sp = 0; sp < S; ++sp) acc += *reinterpret_cast<const f4v*>(ws + (long)sp * M * N + v * 4);
    const int c = (int)((v * 4) % N);
    us4 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = f2bf(act_fwd(act, acc[j] + (bias ? bias[c + j] : 0.f)));
    *reinterpret_cast<us4*>(out + v * 4) = r;
  }
}

// Fraction of CU-slots doing work when `tiles` equal blocks are spread over the
// 256 CUs in rounds (wave quantisation).
static double tile_balance(long tiles) {
  const long cus = 256;
  const long rounds = (tiles + cus - 1) / cus;
  return (double)tiles / (double)(rounds * cus);
}

// 256 x 96 instead of 128 x 128 (forward, both operands K-contiguous, no split): only when the
// 96-wide grid is >= 2 whole rounds and the 128 grid leaves a partial one.  Measured on the
// BERT shapes: QKV (N = 2304) wins; N = 768 (one round of 256 x 96) and N = 3072 (whole
// 128 rounds) lose (profiles/r5_s9/r5s9_gb.log).  CLOUD_AMD_GEMM_256X96=0 turns it off.
static bool use_256x96(const CoreParams& p, int splits) {
  static int en = -1;
  if (en < 0) {
    const char* e = getenv("CLOUD_AMD_GEMM_256X96");
    en = (e && e[0] == '0') ? 0 : 1;
  }
  if (!en || splits != 1 || p.N % 96 || p.M < 4096 || p.stats) return false;
  const long t96 = ((p.M + 255) / 256) * (p.N / 96), t128 = ((p.M + 127) / 128) * ((p.N + 127) / 128);
  return t96 >= 512 && tile_balance(t96) >= 0.999 && tile_balance(t128) < 0.95;
}

// The 256 core pays when its grid fills the chip in (nearly) whole rounds and every block
// has enough K tiles to amortise its 3-tile prologue and its 128-KB epilogue: >= 2 rounds
// at >= 85 % slot use, or exactly whole rounds, and >= 16 K tiles of 32 per block.  (BERT's
// M = 8192 GEMMs get 96-384 tiles -- 1.1-1.5 rounds -- and stay on the 128 core, whose 4
// co-resident blocks per CU absorb the quantisation.)
// Split-K grids (weight gradients) also take it when the caller sized the splits to ONE
// nearly full round of 256 x 256 blocks (ops/raw.py wgrad_into: BERT's FFN / QKV weight
// gradients = 36 x 7 / 27 x 9 blocks).
static bool use_256(const CoreParams& p, int splits) {
  if (core_kind() == 4 || core_kind() == 6) return p.M >= 256 && p.N >= 256;
  if ((core_kind() != 3 && core_kind() != 5) || p.M < 256 || p.N < 256 || p.k_per_split < 512) return false;
  const long t = (long)((p.M + 255) / 256) * ((p.N + 255) / 256) * splits;
  if (splits > 1 && t >= 224 && t <= 256) return true;
  return t >= 256 && (tile_balance(t) >= 0.999 || (t >= 512 && tile_balance(t) >= 0.85));
}

#if CA_EXPERIMENTAL
// 256 x 128 tiles where 256 x 256 tiles do not fill whole rounds but 256 x 128 tiles do
// (BERT-base FFN1 forward / FFN2 input gradient at M = 8192: N = 3072 -> 768 tiles = 3 rounds;
// 256 x 256 gives 384 = 1.5).  Opt-in (CLOUD_AMD_GEMM_256X128=1): measured 669 vs 830 TF/s for
// the 128 core on 8192 x 3072 x 768 and BERT 6,286 / 6,328 vs 6,863 / 6,875 seq/s
// (profiles/r4_s18/) -- one barrier pair per K tile with 16 fragment reads per wave does not
// keep the MFMA pipe as busy as the two-phase 256 x 256 schedule.
static bool use_256x128(const CoreParams& p, int splits) {
  static int en = -1;
  if (en < 0) {
    const char* e = getenv("CLOUD_AMD_GEMM_256X128");
    en = (e && e[0] == '1') ? 1 : 0;
  }
  if (!en || !core_p8() || splits != 1 || p.M < 256 || p.N < 128 || p.K < 512) return false;
  const long t = (long)((p.M + 255) / 256) * ((p.N + 127) / 128);
  return t >= 256 && (tile_balance(t) >= 0.999 || (t >= 512 && tile_balance(t) >= 0.85));
}

// Stream-K (ca_gemm256p8.h) for plain bf16-epilogue GEMMs whose 256 x 256 grid is between
// 3/8 of a round and two rounds of the chip and not whole rounds: BERT-base's M = 8192 forward
// and input-gradient GEMMs (96-384 tiles).  OFF by default (CLOUD_AMD_GEMM_STREAMK=1: those
// shapes, =2: wherever the operands allow -- tests): measured slower than the 128 x 128 core
// it would replace on every BERT shape (bin/gemm_bench, profiles/r5_s4/: QKV forward 57.4 vs
// 42.1 us, FFN2 forward 75.0 vs 59.8, attention output 48.4 vs 19.6) and BERT 5,365 vs 6,866
// seq/s -- the two-phase core's per-iteration rate on short segments plus one 256-KB fp32
// partial store and load per split tile cost more than the last round's idle CUs.
static int g_streamk = -1;
static int streamk_mode() {
  if (g_streamk < 0) {
    const char* e = getenv("CLOUD_AMD_GEMM_STREAMK");
    g_streamk = e ? atoi(e) : 0;
  }
  return g_streamk;
}

static bool use_streamk(const CoreParams& p, int splits) {
  const int mode = streamk_mode();
  if (!mode || !core_p8() || splits != 1 || p.M < 256 || p.N < 256 || p.stats || p.K < 2 * BK) return false;
  if (mode == 2) return true;
  const long t = (long)((p.M + 255) / 256) * ((p.N + 255) / 256);
  const long cus = cu_count();
  return t * 8 >= cus * 3 && t < 2 * cus && tile_balance(t) < 0.999;
}

// Per-stream stream-K workspace: cu_count() fp32 partial tiles (256 KB each) and the tile
// tickets (+1 error word), allocated once per stream and zeroed once -- the owners leave
// their tickets at zero for the next launch, which is ordered after this one on the stream.
struct SkWorkspace {
  float* part = nullptr;
  int* ticket = nullptr;
  int nticket = 0;
};

static int streamk_workspace(hipStream_t s, int tiles, SkParams& S) {
  static SkWorkspace slots[8];
  static hipStream_t keys[8];
  static int used = 0;
  int k = 0;
  while (k < used && keys[k] != s) ++k;
  if (k == used) {
    if (used == 8) return -4;
    keys[used++] = s;
  }
  SkWorkspace& w = slots[k];
  if (!w.part && hipMalloc(&w.part, (size_t)cu_count() * 256 * 256 * 4) != hipSuccess) return -5;
  if (w.nticket < tiles + 1) {
    if (w.ticket) {
      hipStreamSynchronize(s);  // the old tickets may still be in use by a queued launch
      hipFree(w.ticket);
    }
    const int n = tiles + 1 > 1024 ? tiles + 1 : 1024;
    if (hipMalloc(&w.ticket, (size_t)n * 4) != hipSuccess) return -5;
    hipMemsetAsync(w.ticket, 0, (size_t)n * 4, s);
    w.nticket = n;
  }
  S.part = w.part;
  S.ticket = w.ticket;
  S.err_index = w.nticket - 1;
  return 0;
}

#endif  // CA_EXPERIMENTAL

template <int BM, int BN, template <int, int, int> class LA, template <int, int, int> class LB,
          template <int, int, int> class GA, template <int, int, int> class GB, int EPI>
int launch(const CoreParams& p0, int splits, hipStream_t s) {
  CoreParams p = p0;
  p.split_xcd = split_xcd_enabled();
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  // buffer-mode loaders address one block's operand window with 32-bit offsets
  // (ca_mfma_core.h BUF_CAP): rows of a tile (KC) or one split's K range (NC)
  const long span = (long)(p.k_per_split + BK > 256 ? p.k_per_split + BK : 256) * (p.lda > p.ldb ? p.lda : p.ldb) * 2;
  if (use_glds() && span >= (long)BUF_CAP) return -3;
#if CA_EXPERIMENTAL
  if constexpr (BM == 128 && BN == 128 && EPI == EPI_BF16) {
    if (use_streamk(p, splits)) {
      SkParams S{};
      const int t256 = ((p.M + 255) / 256) * ((p.N + 255) / 256);
      const int rc = streamk_workspace(s, t256, S);
      if (rc) return rc;
      S.ipt = (p.K + BK - 1) / BK;
      S.total = t256 * S.ipt;
      // every range non-empty: an empty one would be counted as a contributor by the owner
      const int nwg = (int)(S.total < cu_count() ? S.total : cu_count());
      constexpr bool AK = GA<BM, 1, 256>::KC, BKC = GB<BN, 1, 256>::KC;
      if constexpr (AK && BKC)
        dense_gemm_256p8_sk_kernel<GDenseKC, GDenseKC, EPI><<<nwg, 512, 0, s>>>(p, S);
      else if constexpr (AK && !BKC)
        dense_gemm_256p8_sk_kernel<GDenseKC, GDenseNC, EPI><<<nwg, 512, 0, s>>>(p, S);
      else if constexpr (!AK && !BKC)
        dense_gemm_256p8_sk_kernel<GDenseNC, GDenseNC, EPI><<<nwg, 512, 0, s>>>(p, S);
      else
        return -2;
      CA_LAUNCH_CHECK();
      return 0;
    }
  }
#endif  // CA_EXPERIMENTAL
  if constexpr (BM == 128 && BN == 128 && (EPI == EPI_BF16 || EPI == EPI_F32_PARTIAL || EPI == EPI_BF16_ST)) {
    if (use_256(p, splits)) {
      const int t256 = ((p.M + 255) / 256) * ((p.N + 255) / 256);
      constexpr bool AK = GA<BM, 1, 256>::KC, BKC = GB<BN, 1, 256>::KC;
      if (core_p8()) {
        if constexpr (AK && BKC)
          dense_gemm_256p8_kernel<GDenseKC, GDenseKC, EPI><<<dim3(t256, 1, splits), 512, 0, s>>>(p);
        else if constexpr (AK && !BKC)
          dense_gemm_256p8_kernel<GDenseKC, GDenseNC, EPI><<<dim3(t256, 1, splits), 512, 0, s>>>(p);
        else if constexpr (!AK && !BKC)
          dense_gemm_256p8_kernel<GDenseNC, GDenseNC, EPI><<<dim3(t256, 1, splits), 512, 0, s>>>(p);
        else
          return -2;
        CA_LAUNCH_CHECK();
        return 0;
      }
#if CA_EXPERIMENTAL
      if constexpr (AK && BKC)
        dense_gemm_256_kernel<GDenseKC32, GDenseKC32, EPI><<<dim3(t256, 1, splits), 512, 0, s>>>(p);
      else if constexpr (AK && !BKC)
        dense_gemm_256_kernel<GDenseKC32, GDenseNC, EPI><<<dim3(t256, 1, splits), 512, 0, s>>>(p);
      else if constexpr (!AK && !BKC)
        dense_gemm_256_kernel<GDenseNC, GDenseNC, EPI><<<dim3(t256, 1, splits), 512, 0, s>>>(p);
      else
        return -2;
      CA_LAUNCH_CHECK();
      return 0;
#else
      return -2;  // unreachable: without the experimental build core_p8() holds whenever use_256 does
#endif
    }
    if constexpr (EPI == EPI_BF16 && GA<BM, 1, 256>::KC && GB<BN, 1, 256>::KC) {
      if (use_glds() && use_256x96(p, splits)) {
        const int t = ((p.M + 255) / 256) * (p.N / 96);
        dense_gemm_256x96_kernel<EPI><<<dim3(t, 1, 1), 256, 0, s>>>(p);
        CA_LAUNCH_CHECK();
        return 0;
      }
    }
#if CA_EXPERIMENTAL
    if (use_256x128(p, splits)) {
      const int t = ((p.M + 255) / 256) * ((p.N + 127) / 128);
      constexpr bool AK = GA<BM, 1, 256>::KC, BKC = GB<BN, 1, 256>::KC;
      if constexpr (AK && BKC)
        dense_gemm_256x128_kernel<GDenseKC, GDenseKC, EPI><<<dim3(t, 1, 1), 512, 0, s>>>(p);
      else if constexpr (AK && !BKC)
        dense_gemm_256x128_kernel<GDenseKC, GDenseNC, EPI><<<dim3(t, 1, 1), 512, 0, s>>>(p);
      else
        return -2;
      CA_LAUNCH_CHECK();
      return 0;
    }
#endif  // CA_EXPERIMENTAL
  }
#if CA_EXPERIMENTAL
  if (BN == 128 && core_kind() == 2) {
    dense_gemm_glds8_kernel<BM, BN, GA, GB, EPI><<<dim3(tiles, 1, splits), 512, 0, s>>>(p);
    CA_LAUNCH_CHECK();
    return 0;
  }
#endif
  // K-contiguous operands only (forward GEMMs): the N-contiguous loaders' extra registers
  // make the batched epilogue spill (448-480 B/lane of scratch)
  // Dense-layer epilogues that read memory (act' source, old C for beta) or run the
  // activation: 4 rows' loads in flight per trip instead of one (BERT FFN2 dgrad with
  // GELU': one HBM round trip per staged row otherwise)
  constexpr bool PLAIN = EPI == EPI_BF16;
  if constexpr (PLAIN || (EPI == EPI_BF16_ST && GA<BM, 1, 256>::KC && GB<BN, 1, 256>::KC)) {
    const bool want = !PLAIN || p.dact_src || p.act || p.beta != 0.f;
    if (want && use_glds() && epi_pf()) {
      dense_gemm_glds_pf_kernel<BM, BN, GA, GB, EPI><<<dim3(tiles, 1, splits), 256, 0, s>>>(p);
      CA_LAUNCH_CHECK();
      return 0;
    }
  }
  if (use_glds()) {
    dense_gemm_glds_kernel<BM, BN, GA, GB, EPI><<<dim3(tiles, 1, splits), 256, 0, s>>>(p);
    CA_LAUNCH_CHECK();
    return 0;
  }
  // a single K tile needs no double buffer: half the LDS -> twice the resident blocks
  if (p.k_per_split <= BK)
    dense_gemm_kernel<BM, BN, LA, LB, EPI, 1><<<dim3(tiles, 1, splits), 256, 0, s>>>(p);
  else
    dense_gemm_kernel<BM, BN, LA, LB, EPI, 2><<<dim3(tiles, 1, splits), 256, 0, s>>>(p);
  CA_LAUNCH_CHECK();
  return 0;
}


// 128-wide N tiles unless N is small, or the 128-wide grid would leave a badly
// filled last round (e.g. M=8192, N=768: 384 tiles -> 1.5 rounds) and halving
// the tile width balances it (768 tiles -> 3 full rounds).
static bool want_small_n(const CoreParams& p, int splits) {
  const long tm = (p.M + 127) / 128;
  const long t128 = tm * ((p.N + 127) / 128) * splits, t64 = tm * ((p.N + 63) / 64) * splits;
  return p.N <= 64 || (tile_balance(t128) < 0.8 && tile_balance(t64) > tile_balance(t128) + 0.1);
}

// Transform-A GEMMs (csrc/include/ca_gemm_xa.h): the BN pass that feeds a 1x1 convolution
// runs in that convolution's operand fetch.
template <int BM, int BN, bool BKC, int EPI, int XM>
__global__ void __launch_bounds__(256) xa_gemm_kernel(CoreParams P, XaParams X) {
  mfma_gemm_xa<BM, BN, BKC, EPI, XM>(P, X);
}

// 8-wave form: <= 128 registers per lane so two workgroups (16 waves) fit a CU
template <int BM, int BN, bool BKC, int EPI, int XM>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) xa_gemm8_kernel(CoreParams P,
                                                                                              XaParams X) {
  mfma_gemm_xa<BM, BN, BKC, EPI, XM, 512>(P, X);
}

#if CA_EXPERIMENTAL
// 128 x 256 tiles on 8 waves (2 x 4, wave tile 64 x 64): one workgroup per CU (64 accumulator
// registers per lane on top of the 128 x 128 form's staging).  Measured slower than the 16-wave
// forms (docs/performance.md, round 6): experiment-only (CLOUD_AMD_XA_N256=2)
template <int BM, int BN, bool BKC, int EPI, int XM>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) xa_gemm8w_kernel(CoreParams P,
                                                                                               XaParams X) {
  mfma_gemm_xa<BM, BN, BKC, EPI, XM, 512>(P, X);
}
#endif

// the same tiles with two K tiles' raw operands in flight (coefficients staged in LDS)
template <int BN, bool BKC, int EPI, int XM>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4))) xa_gemm16d_kernel(CoreParams P,
                                                                                                 XaParams X) {
  mfma_gemm_xa_deep<BN, BKC, EPI, XM>(P, X);
}

// 128 x 256 tiles on 16 waves (2 x 8, wave tile 64 x 32: the 128 x 128 8-wave form's registers,
// <= 128 per lane): one workgroup per CU, 16 waves, each A tile transformed once
template <int BM, int BN, bool BKC, int EPI, int XM>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4))) xa_gemm16_kernel(CoreParams P,
                                                                                                XaParams X) {
  mfma_gemm_xa<BM, BN, BKC, EPI, XM, 1024>(P, X);
}

// The 128 x 128 transform-A GEMMs on 8-wave workgroups (default; CLOUD_AMD_XA_WAVES=4: the
// 4-wave form).  ResNet-50 b1024: xa kernels 11.2 -> 10.8 ms/step, 14,614 / 14,617 / 14,560 ->
// 14,668 / 14,650 / 14,582 img/s interleaved (profiles/r4_s20/).
// ... and the 128 x 64 ones (stage 1; CLOUD_AMD_XA_WAVES_N64=0: 4 waves): 85-108 registers;
// 14,775 / 14,784 / 14,767 -> 14,874 / 14,796 / 14,826 img/s interleaved (profiles/r4_s22/)
static bool xa_waves8_n64() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CLOUD_AMD_XA_WAVES_N64");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v != 0;
}
// CLOUD_AMD_XA_N256: transform-A GEMMs with N a multiple of 256 (ResNet-50 stages 3-4: bn3 ->
// conv3 dgrad, bn3 -> next conv1 at N = 256 / 512) on 128 x 256 tiles, so each A tile is read
// and BN-transformed once per 256 columns instead of once per 128.  1: 16-wave workgroups (wave
// tile 64 x 32, <= 128 registers: one per CU); 2: 8 waves (64 x 64, ~190 registers: one per CU
// at half the waves; CLOUD_AMD_BUILD_EXPERIMENTAL builds only); 3 (default): 16 waves with two K
// tiles in flight (mfma_gemm_xa_deep, K <= 2048; else form 1); 0: off (128 x 128 tiles).  The
// two-BN residual epilogue (EPI_BF16_BNR2) keeps the 128-wide tiles: its three statistics rows do
// not fit the 16-wave LDS image.
int g_xa_n256 = -1;
static int xa_n256() {
  if (g_xa_n256 < 0) {
    const char* e = getenv("CLOUD_AMD_XA_N256");
    g_xa_n256 = (e && e[0] >= '0' && e[0] <= '3') ? e[0] - '0' : 3;
  }
  return g_xa_n256;
}
static bool xa_waves8() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CLOUD_AMD_XA_WAVES");
    v = (e && e[0] == '4') ? 0 : 1;
  }
  return v != 0;
}

// two waves per SIMD: two 4-wave or one 8-wave workgroup per CU.  (Two 8-wave workgroups at
// 64 columns would need <= 128 registers per lane: the compiler spilled 135 of them there, 47
// at a 168 budget; 64-row tiles at a 168 budget spilled 19 -- not used.)
template <int EPI, int KS, int NC, int BN, int NT, int BM = 128>
__global__ void __launch_bounds__(NT)
    __attribute__((amdgpu_waves_per_eu(2))) xa_dw_kernel(
        CoreParams P, XaParams X, const bf16_t* Y, long ldy, float* ws, int tiles_per_block) {
  mfma_gemm_xa_dw<EPI, KS, NC, BN, NT, BM>(P, X, Y, ldy, ws, tiles_per_block);
}

// the deep-stream form (ca_gemm_xa.h mfma_gemm_xa_dw_deep): PD = 1 two workgroups per CU,
// PD = 2 / 4 one
template <int EPI, int KS, int PD>
__global__ void __launch_bounds__(256)
    __attribute__((amdgpu_waves_per_eu(PD == 1 ? 2 : 1))) xa_dw_deep_kernel(
        CoreParams P, XaParams X, const bf16_t* Y, long ldy, float* ws, int tiles_per_block) {
  mfma_gemm_xa_dw_deep<EPI, KS, PD>(P, X, Y, ldy, ws, tiles_per_block);
}

// CLOUD_AMD_XA_DW_DEPTH: the K = 256 -> N = 64 kernel (0 = the one-step form above; 1, 2 or 4 =
// the deep form with that many source steps in flight per workgroup).  Stage-1 conv3 shape,
// M = 3.2M (bench/xa_dw_bench.py, profiles/r4_s26/): 1.43 / 0.99 / 1.05 / 1.05 ms with the
// BN-statistics epilogue -- depth 1 at two workgroups per CU is the default.
inline int xa_dw_depth() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CLOUD_AMD_XA_DW_DEPTH");
    v = (e && (e[0] == '0' || e[0] == '1' || e[0] == '2' || e[0] == '4')) ? e[0] - '0' : 1;
  }
  return v;
}

template <int PD>
int xa_dw_deep_launch(const CoreParams& p, const XaParams& x, const bf16_t* Y, long ldy, float* ws, int g, int tpb,
                      hipStream_t s) {
  if (p.bnz) xa_dw_deep_kernel<EPI_BF16_BN, 4, PD><<<g, 256, 0, s>>>(p, x, Y, ldy, ws, tpb);
  else xa_dw_deep_kernel<EPI_BF16, 4, PD><<<g, 256, 0, s>>>(p, x, Y, ldy, ws, tpb);
  CA_LAUNCH_CHECK();
  return 0;
}

template <int KS, int NC, int BN = 64, int NT = 256>
int xa_dw_launch(const CoreParams& p, const XaParams& x, const bf16_t* Y, long ldy, float* ws, int g, int tpb,
                 hipStream_t s) {
  if (p.bnz2) {
    if constexpr (KS == 1) xa_dw_kernel<EPI_BF16_BNR2, KS, NC, BN, NT><<<g, NT, 0, s>>>(p, x, Y, ldy, ws, tpb);
    else return -2;
  } else if (p.res_src) {
    if constexpr (KS == 1) xa_dw_kernel<EPI_BF16_BNR, KS, NC, BN, NT><<<g, NT, 0, s>>>(p, x, Y, ldy, ws, tpb);
    else return -2;
  } else if (p.bnz) {
    xa_dw_kernel<EPI_BF16_BN, KS, NC, BN, NT><<<g, NT, 0, s>>>(p, x, Y, ldy, ws, tpb);
  } else {
    xa_dw_kernel<EPI_BF16, KS, NC, BN, NT><<<g, NT, 0, s>>>(p, x, Y, ldy, ws, tpb);
  }
  CA_LAUNCH_CHECK();
  return 0;
}

template <bool LB, int EPI, int XM>
int xa_launch(const CoreParams& p0, const XaParams& x, hipStream_t s) {
  CoreParams p = p0;
  p.split_xcd = 0;
  const int tm = (p.M + 127) / 128;
  const int n256 = p.N % 256 == 0 ? xa_n256() : 0;
  bool w16 = false;
  if constexpr (EPI != EPI_BF16_BNR2) {  // three 16-wave statistics rows do not fit its LDS image
    if (n256 == 3 && p.K <= XA_DEEP_KMAX) {
      xa_gemm16d_kernel<256, LB, EPI, XM><<<tm * (p.N / 256), 1024, 0, s>>>(p, x);
      w16 = true;
    } else if (n256 == 1 || n256 == 3) {
      xa_gemm16_kernel<128, 256, LB, EPI, XM><<<tm * (p.N / 256), 1024, 0, s>>>(p, x);
      w16 = true;
    }
  }
  bool w8w = false;
#if CA_EXPERIMENTAL
  if (!w16 && n256 == 2) {
    xa_gemm8w_kernel<128, 256, LB, EPI, XM><<<tm * (p.N / 256), 512, 0, s>>>(p, x);
    w8w = true;
  }
#endif
  if (w16 || w8w) {
  } else if (want_small_n(p, 1)) {
    bool w8 = false;
    if constexpr (EPI != EPI_BF16_BNR2) {  // its three statistics rows do not fit the 8-wave LDS image
      if (xa_waves8() && xa_waves8_n64()) {
        xa_gemm8_kernel<128, 64, LB, EPI, XM><<<tm * ((p.N + 63) / 64), 512, 0, s>>>(p, x);
        w8 = true;
      }
    }
    if (!w8) xa_gemm_kernel<128, 64, LB, EPI, XM><<<tm * ((p.N + 63) / 64), 256, 0, s>>>(p, x);
  } else {
    if (xa_waves8()) {
      if constexpr (EPI != EPI_BF16_BNR2)  // its three statistics rows do not fit the 8-wave LDS image
        xa_gemm8_kernel<128, 128, LB, EPI, XM><<<tm * ((p.N + 127) / 128), 512, 0, s>>>(p, x);
      else
        xa_gemm_kernel<128, 128, LB, EPI, XM><<<tm * ((p.N + 127) / 128), 256, 0, s>>>(p, x);
    } else {
      xa_gemm_kernel<128, 128, LB, EPI, XM><<<tm * ((p.N + 127) / 128), 256, 0, s>>>(p, x);
    }
  }
  CA_LAUNCH_CHECK();
  return 0;
}

template <int EPI>
int dispatch(int layout, const CoreParams& p, int splits, hipStream_t s) {
  // stream-K runs on 256 x 256 tiles whatever the 128-tile grid's balance (launch<128, 128>)
#if CA_EXPERIMENTAL
  const bool small_n = !(EPI == EPI_BF16 && use_streamk(p, splits)) && want_small_n(p, splits);
#else
  const bool small_n = want_small_n(p, splits);
#endif
  switch (layout) {
    case 0:
      return small_n ? launch<128, 64, DenseKC, DenseKC, GDenseKC, GDenseKC, EPI>(p, splits, s)
                     : launch<128, 128, DenseKC, DenseKC, GDenseKC, GDenseKC, EPI>(p, splits, s);
    case 1:
      return small_n ? launch<128, 64, DenseKC, DenseNC, GDenseKC, GDenseNC, EPI>(p, splits, s)
                     : launch<128, 128, DenseKC, DenseNC, GDenseKC, GDenseNC, EPI>(p, splits, s);
    case 2:
      // weight gradients with <= 64 output rows (64-channel layers): 64-row tiles, so
      // half of every MFMA is not spent on rows beyond M
      if (p.M <= 64)
        return small_n ? launch<64, 64, DenseNC, DenseNC, GDenseNC, GDenseNC, EPI>(p, splits, s)
                       : launch<64, 128, DenseNC, DenseNC, GDenseNC, GDenseNC, EPI>(p, splits, s);
      return small_n ? launch<128, 64, DenseNC, DenseNC, GDenseNC, GDenseNC, EPI>(p, splits, s)
                     : launch<128, 128, DenseNC, DenseNC, GDenseNC, GDenseNC, EPI>(p, splits, s);
  }
  return -2;
}

CoreParams base_params(const bf16_t* A, long lda, const bf16_t* B, long ldb, void* C, long ldc, int M, int N, int K) {
  CoreParams p{};
  p.A = A; p.lda = lda; p.B = B; p.ldb = ldb; p.C = C; p.ldc = ldc;
  p.M = M; p.N = N; p.K = K; p.k_per_split = K;
  return p;
}

}  // namespace

extern "C" {

int ca_dgrad_gemm(int layout, const bf16_t* A, long lda, const bf16_t* B, long ldb, bf16_t* C, long ldc, int M, int N,
                  int K, float beta, const bf16_t* res_src, const uint8_t* res_mask, const bf16_t* bnz,
                  const uint8_t* bnmask, float* stats, hipStream_t s, const bf16_t* bnz2, float* stats2,
                  int par_s, int par_h, int par_w);

// Select the GEMM core for this process (values as CLOUD_AMD_GEMM_CORE above); returns
// the previous one.
// Stream-K mode (CLOUD_AMD_GEMM_STREAMK: 0 off, 1 auto, 2 wherever allowed); returns the previous.
// -1: stream-K is not in this build (CLOUD_AMD_BUILD_EXPERIMENTAL=1 builds it)
int ca_gemm_set_streamk(int mode) {
#if CA_EXPERIMENTAL
  const int prev = streamk_mode();
  if (mode >= 0 && mode <= 2) g_streamk = mode;
  return prev;
#else
  (void)mode;
  return -1;
#endif
}

int ca_gemm_experimental_built() { return CA_EXPERIMENTAL; }

// -1: the requested core is not in this build (kinds 2-4 need CLOUD_AMD_BUILD_EXPERIMENTAL=1)
int ca_gemm_set_core(int kind) {
  const int prev = core_kind();
  if (!CA_EXPERIMENTAL && kind >= 2 && kind <= 4) return -1;
  if (kind >= 0 && kind <= 6) g_core_kind = kind;
  return prev;
}

// Transform-A tiles for N % 256 == 0 (values as CLOUD_AMD_XA_N256); returns the previous mode.
int ca_gemm_set_xa_n256(int mode) {
  const int prev = xa_n256();
  if (mode == 2 && !CA_EXPERIMENTAL) return -1;  // the 8-wave form is experiment-only
  if (mode >= 0 && mode <= 3) g_xa_n256 = mode;
  return prev;
}

int ca_splitk_bias_act(const float* ws, int splits, long M, int N, const float* bias, int act, bf16_t* out,
                       hipStream_t s) {
  if (N % 4 || M <= 0) return -1;
  splitk_bias_act_kernel<<<ca_stream_grid(M * N / 4, 256), 256, 0, s>>>(ws, splits, M, N, bias, act, out);
  CA_LAUNCH_CHECK();
  return 0;
}

int ca_splitk_reduce(const float* ws, int splits, long MN, void* out, int out_bf16, float beta, hipStream_t s) {
  if (MN % 4) return -3;
  const long n4 = MN / 4;
  if (n4 >= 64L * 512) {  // large output: streaming column kernel (same rule in gradfin.hip)
    const int g = (int)((n4 + 255) / 256);
    if (out_bf16) splitk_reduce_cols_kernel<true><<<g, 256, 0, s>>>(ws, splits, MN, out, beta);
    else splitk_reduce_cols_kernel<false><<<g, 256, 0, s>>>(ws, splits, MN, out, beta);
    CA_LAUNCH_CHECK();
    return 0;
  }
  int CB = 16;
  if (n4 < 16L * 512) CB = 4;
  const int grid = (int)((n4 + CB - 1) / CB);
  if (out_bf16) splitk_reduce_kernel<true><<<grid, 256, 0, s>>>(ws, splits, MN, out, beta, CB);
  else splitk_reduce_kernel<false><<<grid, 256, 0, s>>>(ws, splits, MN, out, beta, CB);
  CA_LAUNCH_CHECK();
  return 0;
}

// C = A*B (+ beta*C) in bf16.  stats != null -> per-128-row-tile column [sum|sumsq] partials.
int ca_gemm_bf16(int layout, const bf16_t* A, long lda, const bf16_t* B, long ldb, bf16_t* C, long ldc,
                 int M, int N, int K, float* stats, float beta, hipStream_t s) {
  if (M <= 0 || N < 8 || N % 8 != 0 || K % 8 != 0 || (layout == 2 && M % 8 != 0)) return -1;
  CoreParams p = base_params(A, lda, B, ldb, C, ldc, M, N, K);
  p.stats = stats;
  p.beta = beta;
  if (!stats && layout == 0 && prw_kind(M, N, K, lda, ldb, ldc, false) == 2) return prw_launch(2, p, s);
  if (stats && layout == 0) {  // forward 1x1 conv feeding a BatchNorm: register-accumulated statistics
    const int kind = prw_kind(M, N, K, lda, ldb, ldc, true);
    if (kind && prw_grid(kind, M) > 0) return prw_launch(kind, p, s);  // one partial row per workgroup / range
    return want_small_n(p, 1) ? launch<128, 64, DenseKC, DenseKC, GDenseKC, GDenseKC, EPI_BF16_ST>(p, 1, s)
                              : launch<128, 128, DenseKC, DenseKC, GDenseKC, GDenseKC, EPI_BF16_ST>(p, 1, s);
  }
  return dispatch<EPI_BF16>(layout, p, 1, s);
}

// Rows of the [rows][2][N] statistics partials ca_gemm_bf16(layout 0, stats != null) writes:
// one per workgroup on the persistent core, one per 128 GEMM rows otherwise.
int ca_gemm_stat_rows(int M, int N, int K, long lda, long ldb, long ldc) {
  const int kind = prw_kind(M, N, K, lda, ldb, ldc, true);
  return (kind && prw_grid(kind, M) > 0) ? prw_stat_rows(kind, M) : (M + 127) / 128;
}

// Input-gradient GEMM (NN: dX = dY W) whose output feeds a BatchNorm(+ReLU) backward:
// the epilogue also writes per-128-row-tile column partials [sum g | sum g*z] into
// `stats` ([tiles_m][2][N]), g = C * relu'(mask), z = the BN input (ld = ldc) -- the
// BN backward then skips its own reduction pass over dy and z.
int ca_gemm_bf16_bnstats(int layout, const bf16_t* A, long lda, const bf16_t* B, long ldb, bf16_t* C, long ldc,
                         int M, int N, int K, float beta, const bf16_t* bnz, const uint8_t* bnmask, float* stats,
                         hipStream_t s) {
  return ca_dgrad_gemm(layout, A, lda, B, ldb, C, ldc, M, N, K, beta, nullptr, nullptr, bnz, bnmask, stats, s, nullptr,
                       nullptr, 0, 0, 0);
}

// Input-gradient GEMM (NN) with the two backward epilogue options of a ResNet block:
//   res_src [+ res_mask]: C = A*B + beta * relu'(res_mask) * res_src -- the block's
//                         identity-path gradient gated from the output gradient on the
//                         fly (never materialised);
//   bnz / bnmask / stats: BN-backward statistics of C for the BN that consumes it;
//   bnz2 / stats2 (with res_src): the same for a second BN fed by the same gated gradient.
int ca_dgrad_gemm(int layout, const bf16_t* A, long lda, const bf16_t* B, long ldb, bf16_t* C, long ldc, int M, int N,
                  int K, float beta, const bf16_t* res_src, const uint8_t* res_mask, const bf16_t* bnz,
                  const uint8_t* bnmask, float* stats, hipStream_t s, const bf16_t* bnz2, float* stats2,
                  int par_s, int par_h, int par_w) {
  if (M <= 0 || N < 8 || N % 8 != 0 || K % 8 != 0 || layout != 1 || (bnz && !stats)) return -1;
  if (bnz2 && (!bnz || !stats2 || !res_src)) return -1;
  // par_s > 1: old C stored only at pixels (h, w) both multiples of par_s of an [*, par_h, par_w]
  // image (rows are its NHWC pixels, ldc its channels): the other rows' beta term is zero
  if (par_s > 1 && (par_h <= 0 || par_w <= 0 || M % ((long)par_h * par_w) != 0 || res_src)) return -1;
  CoreParams p = base_params(A, lda, B, ldb, C, ldc, M, N, K);
  p.beta = beta;
  p.res_src = res_src;
  p.res_mask = res_mask;
  if (par_s > 1 && beta != 0.f) {
    p.bpar_s = par_s;
    p.div_bpw = make_fastdiv(par_w);
    p.div_bph = make_fastdiv(par_h);
  }
  if (!bnz) return dispatch<EPI_BF16>(layout, p, 1, s);
  p.stats = stats;
  p.bnz = bnz;
  p.bnmask = bnmask;
  if (bnz2) {
    p.bnz2 = bnz2;
    p.stats2 = stats2;
    return want_small_n(p, 1) ? launch<128, 64, DenseKC, DenseNC, GDenseKC, GDenseNC, EPI_BF16_BNR2>(p, 1, s)
                              : launch<128, 128, DenseKC, DenseNC, GDenseKC, GDenseNC, EPI_BF16_BNR2>(p, 1, s);
  }
  if (res_src)
    return want_small_n(p, 1) ? launch<128, 64, DenseKC, DenseNC, GDenseKC, GDenseNC, EPI_BF16_BNR>(p, 1, s)
                              : launch<128, 128, DenseKC, DenseNC, GDenseKC, GDenseNC, EPI_BF16_BNR>(p, 1, s);
  return want_small_n(p, 1) ? launch<128, 64, DenseKC, DenseNC, GDenseKC, GDenseNC, EPI_BF16_BN>(p, 1, s)
                            : launch<128, 128, DenseKC, DenseNC, GDenseKC, GDenseNC, EPI_BF16_BN>(p, 1, s);
}

// Dense-layer GEMM with the fused epilogue: C = act(A*B + bias) (+ beta*C),
// pre-activation kept in `preact` when given; backward form: C = (A*B) * act'(dact_src).
int ca_gemm_ex(int layout, const bf16_t* A, long lda, const bf16_t* B, long ldb, bf16_t* C, long ldc, int M, int N,
               int K, float* stats, float beta, const float* bias, int act, bf16_t* preact, const bf16_t* dact_src,
               long ld_aux, hipStream_t s) {
  if (M <= 0 || N < 8 || N % 8 != 0 || K % 8 != 0 || (layout == 2 && M % 8 != 0)) return -1;
  if ((preact || dact_src) && ld_aux % 8 != 0) return -1;
  CoreParams p = base_params(A, lda, B, ldb, C, ldc, M, N, K);
  p.stats = stats;
  p.beta = beta;
  p.bias = bias;
  p.act = act;
  p.preact = preact;
  p.dact_src = dact_src;
  p.ld_aux = ld_aux;
  return dispatch<EPI_BF16>(layout, p, 1, s);
}

// Transform-A GEMM (ca_gemm_xa.h).  layout 0 (NT, forward 1x1 conv: B = W [N][K]) with
// mode XA_BN_RELU / XA_BN_RES_RELU / XA_BN_RESBN_RELU and the BN-forward statistics epilogue
// when `stats`;
// layout 1 (NN, input gradient: B = W [K][N]) with mode XA_BN_BWD and the dgrad epilogues of
// ca_dgrad_gemm (BN-backward statistics bnz/bnmask/stats, residual-gated beta res_src/res_mask,
// second BN bnz2/stats2).  The A operand is X(src0, src1, mask_in; c0, c1, c2) [M][K] with row
// stride lda; `side` / `mask_out` receive the transformed A and (forward) its ReLU bitmask.
int ca_gemm_xa(int layout, int mode, const bf16_t* src0, const bf16_t* src1, const uint8_t* mask_in,
               const float* c0, const float* c1, const float* c2, const float* c3, bf16_t* side, uint8_t* mask_out,
               long lda,
               const bf16_t* B, long ldb, bf16_t* C, long ldc, int M, int N, int K, float beta,
               const bf16_t* res_src, const uint8_t* res_mask, const bf16_t* bnz, const uint8_t* bnmask,
               float* stats, const bf16_t* bnz2, float* stats2, hipStream_t s) {
  if (M <= 0 || N < 8 || N % 8 != 0 || K < 8 || K % 8 != 0 || lda % 8 != 0 || !src0 || !c0 || !c1) return -1;
  if ((mode == XA_BN_RES_RELU && !src1) || (mode == XA_BN_BWD && (!src1 || !c2))) return -1;
  if (mode == XA_BN_RESBN_RELU && (!src1 || !c2 || !c3)) return -1;
  if ((bnz && !stats) || (bnz2 && (!bnz || !stats2 || !res_src))) return -1;
  CoreParams p = base_params(src0, lda, B, ldb, C, ldc, M, N, K);
  p.beta = beta;
  XaParams x{src0, src1, mask_in, c0, c1, c2, c3, side, mask_out};
  if (layout == 0) {
    if (beta != 0.f || res_src || bnz) return -1;
    p.stats = stats;
    if (mode == XA_BN_RELU)
      return stats ? xa_launch<true, EPI_BF16_ST, XA_BN_RELU>(p, x, s) : xa_launch<true, EPI_BF16, XA_BN_RELU>(p, x, s);
    if (mode == XA_BN_RES_RELU)
      return stats ? xa_launch<true, EPI_BF16_ST, XA_BN_RES_RELU>(p, x, s)
                   : xa_launch<true, EPI_BF16, XA_BN_RES_RELU>(p, x, s);
    if (mode == XA_BN_RESBN_RELU)
      return stats ? xa_launch<true, EPI_BF16_ST, XA_BN_RESBN_RELU>(p, x, s)
                   : xa_launch<true, EPI_BF16, XA_BN_RESBN_RELU>(p, x, s);
    return -2;
  }
  if (layout != 1 || mode != XA_BN_BWD) return -2;
  p.res_src = res_src;
  p.res_mask = res_mask;
  if (!bnz) return xa_launch<false, EPI_BF16, XA_BN_BWD>(p, x, s);
  p.stats = stats;
  p.bnz = bnz;
  p.bnmask = bnmask;
  if (bnz2) {
    p.bnz2 = bnz2;
    p.stats2 = stats2;
    return xa_launch<false, EPI_BF16_BNR2, XA_BN_BWD>(p, x, s);
  }
  if (res_src) return xa_launch<false, EPI_BF16_BNR, XA_BN_BWD>(p, x, s);
  return xa_launch<false, EPI_BF16_BN, XA_BN_BWD>(p, x, s);
}

// XA_BN_BWD input gradient of a stride-s 1x1 / pad-0 convolution (a ResNet projection shortcut):
// dz = A*(dy*relu'(mask)) + B*z + D is produced in the operand fetch (and written to `side`, the
// weight gradient's operand), dX = dz W goes to the one non-empty output-parity class of
// dx[Nb, H, W, ldc] -- GEMM row (n, qy, qx) to pixel (n, s*qy, s*qx) -- the other pixels are
// left unwritten (the caller's next input-gradient GEMM reads them as zeros: CoreParams::bpar_s).
// M must be Nb * ceil(H/s) * ceil(W/s).
int ca_gemm_xa_bwd_strided(const bf16_t* src0, const bf16_t* src1, const uint8_t* mask_in, const float* c0,
                           const float* c1, const float* c2, bf16_t* side, long lda, const bf16_t* B, long ldb,
                           bf16_t* C, long ldc, int M, int N, int K, int Nb, int H, int W, int stride, hipStream_t s) {
  if (M <= 0 || N < 8 || N % 8 != 0 || K < 8 || K % 8 != 0 || lda % 8 != 0 || !src0 || !src1 || !c0 || !c1 || !c2)
    return -1;
  const int Hq = (H + stride - 1) / stride, Wq = (W + stride - 1) / stride;
  if (stride < 2 || (long)Nb * Hq * Wq != M) return -1;
  CoreParams p = base_params(src0, lda, B, ldb, C, ldc, M, N, K);
  p.rowmap = 1;
  p.dg_py = 0;
  p.dg_px = 0;
  p.Nb = Nb;
  p.H = H;
  p.W = W;
  p.sh = stride;
  p.sw = stride;
  p.Hq = Hq;
  p.Wq = Wq;
  p.div_hq = make_fastdiv(Hq);
  p.div_wq = make_fastdiv(Wq);
  XaParams x{src0, src1, mask_in, c0, c1, c2, nullptr, side, nullptr};
  return xa_launch<false, EPI_BF16, XA_BN_BWD>(p, x, s);
}

// XA_BN_BWD input gradient with the weight gradient in the same pass (ca_gemm_xa.h
// mfma_gemm_xa_dw).  Shapes: N == 64 with K in {64, 128, 256} (stage-1 conv3), K == 64 with
// N == 256 (stage-1 conv1), N == 128 with K == 512 (stage-2 conv3, 8-wave workgroups); the dgrad epilogues of ca_gemm_xa layout 1 (BN statistics bnz/bnmask/
// stats, residual-gated res_src/res_mask, second BN bnz2/stats2 -- the last two at K == 64
// only) and a plain beta accumulate into C.  `blocks` workgroups each own a contiguous range
// of 128-row tiles and write one fp32 dW slab ([K][N]) into ws (blocks * K * N floats);
// dw (bf16 when dw_bf16, else fp32, [K][N]) = sum of the slabs + dw_beta * dw.  dz is never
// written.  Returns the workgroup count used (>= 1) or a negative code.
int ca_gemm_xa_dw(const bf16_t* src0, const bf16_t* src1, const uint8_t* mask_in, const float* c0, const float* c1,
                  const float* c2, long lda, const bf16_t* B, long ldb, bf16_t* C, long ldc, int M, int N, int K,
                  float beta, const bf16_t* res_src, const uint8_t* res_mask, const bf16_t* bnz,
                  const uint8_t* bnmask, float* stats, const bf16_t* bnz2, float* stats2, const bf16_t* Y, long ldy,
                  void* dw, int dw_bf16, float dw_beta, float* ws, int blocks, hipStream_t s) {
  if (M <= 0 || lda % 8 != 0 || ldy % 8 != 0 || ldc % 8 != 0 || !src0 || !src1 || !c0 || !c1 || !c2 || !Y || !dw ||
      !ws || blocks <= 0)
    return -1;
  if ((bnz && !stats) || (bnz2 && (!bnz || !stats2 || !res_src))) return -1;
  CoreParams p = base_params(src0, lda, B, ldb, C, ldc, M, N, K);
  p.beta = beta;
  p.res_src = res_src;
  p.res_mask = res_mask;
  p.bnz = bnz;
  p.bnmask = bnmask;
  p.stats = stats;
  p.bnz2 = bnz2;
  p.stats2 = stats2;
  XaParams x{src0, src1, mask_in, c0, c1, c2, nullptr, nullptr, nullptr};
  const int tiles = (M + 127) / 128;
  const int depth = (N == 64 && K == 256) ? xa_dw_depth() : 0;
  static int w8 = -1;  // CLOUD_AMD_XA_DW_WAVES=8: one 8-wave workgroup per CU (one-step form)
  if (w8 < 0) {
    const char* e = getenv("CLOUD_AMD_XA_DW_WAVES");
    w8 = (e && e[0] == '8') ? 1 : 0;
  }
  // deep form: beta 0, no residual / second BN, statistics exactly with a BN input
  bool deep = depth > 0 && !w8 && beta == 0.f && !res_src && !bnz2 && (bnz != nullptr) == (stats != nullptr);
  {  // the deep form reads each tensor through ONE buffer window over a workgroup's tile range
    const int b = (depth >= 2 && blocks > cu_count()) ? cu_count() : blocks;
    const long rows = (long)((tiles + b - 1) / b) * 128;
    long ld = lda > ldy ? lda : ldy;
    if (ldc > ld) ld = ldc;
    if (rows * ld * 2 >= (long)BUF_CAP) deep = false;
  }
  // deep forms at one workgroup per CU: one tile range per CU
  if (deep && depth >= 2 && blocks > cu_count()) blocks = cu_count();
  const int tpb = (tiles + blocks - 1) / blocks;
  const int g = (tiles + tpb - 1) / tpb;
  int rc;
  if (N == 64 && K == 64) rc = xa_dw_launch<1, 1>(p, x, Y, ldy, ws, g, tpb, s);
  else if (N == 64 && K == 128) rc = xa_dw_launch<2, 1>(p, x, Y, ldy, ws, g, tpb, s);
  else if (N == 64 && K == 256) {
    if (deep && depth == 1) rc = xa_dw_deep_launch<1>(p, x, Y, ldy, ws, g, tpb, s);
    else if (deep && depth == 2) rc = xa_dw_deep_launch<2>(p, x, Y, ldy, ws, g, tpb, s);
    else if (deep) rc = xa_dw_deep_launch<4>(p, x, Y, ldy, ws, g, tpb, s);
    else rc = w8 ? xa_dw_launch<4, 1, 64, 512>(p, x, Y, ldy, ws, g, tpb, s) : xa_dw_launch<4, 1>(p, x, Y, ldy, ws, g, tpb, s);
  }
  else if (K == 64 && N == 256) rc = xa_dw_launch<1, 4>(p, x, Y, ldy, ws, g, tpb, s);
  else if (N == 128 && K == 512) rc = xa_dw_launch<8, 1, 128, 512>(p, x, Y, ldy, ws, g, tpb, s);
  else return -1;
  if (rc < 0) return rc;
  rc = ca_splitk_reduce(ws, g, (long)K * N, dw, dw_bf16, dw_beta, s);
  return rc < 0 ? rc : g;
}

int ca_gemm_splitk_effective(int K, int splits) {
  int kps = (K / splits + BK - 1) / BK * BK;
  if (kps < BK) kps = BK;
  return (K + kps - 1) / kps;
}

// Split-K GEMM into fp32 slabs ws[splits][M][N] + deterministic reduction into
// `out` (bf16 if out_bf16 else fp32): out = sum + beta*out.  out_bf16 < 0: slabs only.
int ca_gemm_splitk(int layout, const bf16_t* A, long lda, const bf16_t* B, long ldb, void* out, int out_bf16,
                   float beta, int M, int N, int K, int splits, float* ws, hipStream_t s) {
  if (M <= 0 || N < 8 || N % 8 != 0 || (layout == 2 && M % 8 != 0)) return -1;
  int kps = (K / splits + BK - 1) / BK * BK;
  if (kps < BK) kps = BK;
  splits = (K + kps - 1) / kps;
  CoreParams p = base_params(A, lda, B, ldb, ws, N, M, N, K);
  p.k_per_split = kps;
  p.split_stride = (long)M * N;
  int rc = dispatch<EPI_F32_PARTIAL>(layout, p, splits, s);
  if (rc || out_bf16 < 0) return rc;  // out_bf16 < 0: slabs only, the caller reduces them (gradfin.hip)
  return ca_splitk_reduce(ws, splits, (long)M * N, out, out_bf16, beta, s);
}

}  // extern "C"
