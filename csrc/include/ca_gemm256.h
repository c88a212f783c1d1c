// 256 x 256 MFMA GEMM core for large GEMMs (gfx950 / CDNA4): 8 waves in two groups that
// alternate compute and load roles barrier by barrier, over a 4-stage LDS-DMA ring.
//
//   C[M,N] = sum_k A(m,k) * B(k,n)     bf16 operands, fp32 accumulation
//
// Geometry: one 512-thread workgroup per CU (2 waves per SIMD), tile 256 x 256, waves 2 (M)
// x 4 (N) with a 128 x 64 wave tile (8 x 4 fragments of v_mfma_f32_16x16x32_bf16).  The K
// tile is 32 deep; the LDS holds a ring of 4 stages of [A 256x32 | B 256x32] (32 KB each).
// Wave group 1 (waves 4-7) runs one barrier behind group 0, so on every SIMD one wave
// multiplies while its partner reads LDS and issues LDS-DMA (MI355X_MICROARCH.md "Two waves
// per SIMD").  Every K tile is ONE phase per wave: {R: 12 fragment reads (A 8, B 4) + the 4
// LDS-DMA pieces of tile t+3} barrier {M: 32 MFMAs} barrier.  Pieces are issued three tiles
// (six barrier intervals, ~2,000 cycles) ahead of their use and retired by a counted
// vmcnt(8) -- two tiles stay in flight, the loop never drains to zero -- and a stage is
// refilled only after the barrier that follows its last read.
//
// How it was chosen (MI355X, bin/gemm_bench + rocprofv3 counters; docs/performance.md,
// "GEMM core, round 3"): uniform [-1,1) operands, bf16 out,
//                               4096^3 TF/s   8192^3 TF/s   MFMA busy @8192^3   clock
//   128^2, 4 waves, 1 stage (old)    904          845            0.47            1.71 GHz
//   this core                      1126-1148    1166-1175        0.66            1.67-1.71
//   hipBLASLt (torch.mm)             1418         1479            0.885           1.61
// Rejected on the way (all numerically correct, all slower): the same ping-pong with BK = 64
// and 16-MFMA phases (1028-1063 / 1112; read segments longer than the partner's MFMAs),
// and four 4-wave 128x128-per-wave designs with 256 AGPR accumulators -- register staging
// at the tile head (822 / 947: the LDS write path stalls), LDS-DMA spread over the MFMA
// groups (943-976 / 1080-1087: ~60 wave cycles per piece on the only wave of a SIMD),
// register staging spread over the groups (900 / 1030: LDS issue stalls), and the
// global_load_lds form of the DMA (844 / 1008).  hipBLASLt's kernels are 4-wave persistent
// ones with shape-tuned macro tiles (256x160, 192x256, 192x128).
//
// K-contiguous tiles are [rows][32] with 64-B rows; the st_16x32 swizzle (16-B chunk ^=
// 2 * bit 3 of the row) makes the ds_read_b128 fragment reads conflict-free and is applied
// on the DMA source side (lane-linear LDS image, cdna_hip_programming.md rule 21).
// N-contiguous tiles are [32 k][256] read with ds_read_b64_tr_b16 exactly as in the BK = 64
// cores (GDenseNC loaders: 2 rounds of 16 k rows).
#pragma once
#include <type_traits>

#include "ca_mfma_core.h"

namespace ca {

__device__ __forceinline__ void bar256() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void lgkm_wait0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Tile walk of the persistent / data-parallel 256 cores.  Tiles are dealt to XCDs in
// contiguous ranges (xcd_remap), and inside a range they run in groups of GM tile rows,
// column-major within the group, so the blocks of one XCD share A row panels and B
// column panels in their L2.
__device__ __forceinline__ void tile256_coords(int id, int tiles_m, int tiles_n, int& tm, int& tn) {
  constexpr int GM = 4;
  const int per_group = GM * tiles_n;
  const int g = id / per_group;
  const int first_m = g * GM;
  const int rows = (tiles_m - first_m) < GM ? (tiles_m - first_m) : GM;
  const int r = id - g * per_group;
  tm = first_m + r % rows;
  tn = r / rows;
}

__device__ __forceinline__ int kc32_swz(int row) { return ((row >> 3) & 1) << 1; }

// Dense K-contiguous operand, 64-B (32-element) K tiles: X[r][k] at p[r*ld + k].
// Chunk i of thread tid: tile row (tid >> 2) + i * (NT / 4), 16-B slot tid & 3.
template <int R, int CPT, int NT>
struct GDenseKC32 {
  static constexpr bool KC = true, BUF = true;
  const bf16_t* sbase;
  uint32_t nrec, roff, ldb2;
  int col, K;
  __device__ GDenseKC32(const CoreParams& P, bool isA, int r0, int tid) {
    const bf16_t* p = isA ? P.A : P.B;
    const long ld = isA ? P.lda : P.ldb;
    const int rows = isA ? P.M : P.N;
    K = P.K;
    const int row = tid >> 2;
    col = ((tid & 3) ^ kc32_swz(row)) << 3;
    sbase = p + (long)r0 * ld;
    nrec = buf_span((long)(rows - r0) * ld * 2);
    ldb2 = (uint32_t)(ld * 2);
    roff = (uint32_t)((row * ld + col) * 2);
  }
  __device__ __forceinline__ uint32_t off(int i, int k0) const {
    const uint32_t o = roff + (uint32_t)(i * (NT / 4)) * ldb2 + (uint32_t)k0 * 2u;
    return (k0 + col < K) ? o : nrec;
  }
};

template <int R, bool KC>
__device__ __forceinline__ bf16x8 read_frag32(const short* lds, int r0, int lane) {
  if constexpr (KC) {
    const int row = r0 + (lane & 15);
    const int pc = (lane >> 4) ^ kc32_swz(row);
    s8v v = *reinterpret_cast<const s8v*>(lds + row * 32 + pc * 8);
    return __builtin_bit_cast(bf16x8, v);
  } else {
    return read_frag_sw<R, false>(lds, r0, 0, lane);
  }
}

template <template <int, int, int> class LAT, template <int, int, int> class LBT, int EPI, bool STAMP = false>
__device__ __forceinline__ void mfma_gemm_256(const CoreParams& P) {
  constexpr int BM = 256, BN = 256, WN = 4, NT = 512, KT = 32, NS = 4;
  constexpr int FM = 8, FN = 4;
  constexpr int A_ELEMS = BM * KT, B_ELEMS = BN * KT;
  constexpr int STAGE = A_ELEMS + B_ELEMS;
  constexpr int SMEM = NS * STAGE;
  static_assert(SMEM >= BM * EpiLayout<BN>::LD, "C staging must fit the ring");
  constexpr int CPA = A_ELEMS / 8 / NT, CPB = B_ELEMS / 8 / NT;
  static_assert(CPA == 2 && CPB == 2, "two pieces per operand and tile");
  using LA = LAT<BM, CPA, NT>;
  using LB = LBT<BN, CPB, NT>;
  constexpr bool A_KC = LA::KC, B_KC = LB::KC;
  __shared__ __attribute__((aligned(16))) short smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int grp = __builtin_amdgcn_readfirstlane(wave) >> 2;
  const int tiles_m = (P.M + BM - 1) / BM, tiles_n = (P.N + BN - 1) / BN;
  const BlkPos bp = blk_pos(P);
  int tm, tn;
  tile256_coords(bp.tile, tiles_m, tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = bp.split * P.k_per_split;
  int kend = kbeg + P.k_per_split;
  if (kend > P.K) kend = P.K;
  const int nk = (kend - kbeg + KT - 1) / KT;

  const LA la(P, true, m0, tid);
  const LB lb(P, false, n0, tid);
  const auto ra = loader_rsrc(la);
  const auto rb = loader_rsrc(lb);

  f4v acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int t) {
    short* base = smem + (t & (NS - 1)) * STAGE;
    const int k0 = kbeg + t * KT;
#pragma unroll
    for (int i = 0; i < CPA; ++i) CA_DMA_CHUNK(LA, la, ra, i, k0, base + (i * NT + wave * 64) * 8);
#pragma unroll
    for (int i = 0; i < CPB; ++i) CA_DMA_CHUNK(LB, lb, rb, i, k0, base + A_ELEMS + (i * NT + wave * 64) * 8);
  };

  unsigned long long st[4];
  const int ts = nk / 2;
  bf16x8 af[FM], bfr[FN];
  const int ar0 = wm * (BM / 2), bc0 = wn * (BN / WN);

  if (nk > 0) issue(0);
  if (nk > 1) issue(1);
  if (nk > 2) issue(2);
  if (nk > 2) vm_wait<8>();
  else if (nk > 1) vm_wait<4>();
  else vm_wait<0>();
  bar256();
  if (grp == 1) bar256();

  for (int t = 0; t < nk; ++t) {
    const short* As = smem + (t & (NS - 1)) * STAGE;
    const short* Bs = As + A_ELEMS;
    if constexpr (STAMP) {
      if (t == ts) st[0] = __builtin_amdgcn_s_memtime();
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) af[i] = read_frag32<BM, A_KC>(As, ar0 + i * 16, lane);
#pragma unroll
    for (int j = 0; j < FN; ++j) bfr[j] = read_frag32<BN, B_KC>(Bs, bc0 + j * 16, lane);
    if (t + 3 < nk) {
      issue(t + 3);
      vm_wait<8>();
    } else if (t + 2 < nk) {
      vm_wait<4>();
    } else {
      vm_wait<0>();
    }
    lgkm_wait0();
    if constexpr (STAMP) {
      if (t == ts) st[1] = __builtin_amdgcn_s_memtime();
    }
    bar256();
    if constexpr (STAMP) {
      if (t == ts) st[2] = __builtin_amdgcn_s_memtime();
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    if constexpr (STAMP) {
      if (t == ts) st[3] = __builtin_amdgcn_s_memtime();
    }
    bar256();
  }
  if (grp == 0) bar256();
  if constexpr (STAMP) {
    if (lane == 0 && P.stamps) {
      unsigned long long* o = P.stamps + ((long)blockIdx.x * 8 + wave) * 17;
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = st[k];
    }
  }
  __syncthreads();
  gemm_epilogue<BM, BN, 2, WN, EPI, SMEM>(P, acc, smem, m0, n0, tm, tid);
}

}  // namespace ca
