// 256 x 256 pipelined MFMA GEMM core (gfx950 / CDNA4) -- the "v3" core.
//
//   C[M,N] = sum_k A(m,k) * B(k,n)     bf16 operands, fp32 accumulation
//
// Geometry: one 512-thread workgroup (8 waves, 2 per SIMD) per CU, tile 256 x 256,
// BK = 64, two LDS stages of [A 256x64 | B 256x64] (128 KB).  Waves are 2 (M) x 4 (N)
// with a 128 x 64 wave tile: 8 x 4 accumulator fragments of v_mfma_f32_16x16x32_bf16.
//
// Why this shape (measured on MI355X, docs/performance.md): the 4-wave 128^2 core keeps
// the matrix pipes ~49 % busy because each K step is load -> wait -> barrier -> MFMA and
// only co-resident blocks hide the wait.  Here every wave owns a SIMD together with one
// partner and the two alternate roles barrier by barrier (MI355X_MICROARCH.md "Two waves
// per SIMD"): wave group 1 (waves 4-7) runs one barrier behind group 0, so in every
// barrier interval one wave of each SIMD multiplies while its partner reads LDS and issues
// LDS-DMA.
//
// K tile t is four phases, each {R: LDS reads + 2 LDS-DMA pieces} barrier {M: 16 MFMAs}
// barrier, over (k half, M half) of the wave tile:
//
//   phase  reads              MFMAs            DMA issued (8 pieces per tile, 2 per phase)
//   q0     A(mh0,k0) B(k0) 8  acc rows 0-63    B pair Y of tile t+1    + vmcnt: A pair P2(t)
//   q1     A(mh1,k0)       4  acc rows 64-127  A pair P1 of tile t+1
//   q2     A(mh0,k1) B(k1) 8  acc rows 0-63    A pair P2 of tile t+1
//   q3     A(mh1,k1)       4  acc rows 64-127  B pair X of tile t+2    + vmcnt: tile t+1 minus P2
//
// Reads are spread 8/4/8/4 (the 128^2-quadrant order would read 12/12/0/0 and make the read
// segment longer than the partner's 16-MFMA segment).  A "pair" is two DMA rounds; round i
// of an operand is chunk i of every thread (KC operands: 64 rows x 128 B; NC operands: 16 k
// rows x 512 B).  Pairs are chosen so every DMA lands in LDS bytes whose last reader has
// passed a barrier (WAR) and every read follows the issuing waves' counted vmcnt plus a
// barrier (RAW; cdna_hip_programming.md "Read a staged buffer one phase AFTER the wait"):
//   A P1 = rows of M half 0 of both wave groups (KC rounds 0,2) | k rows 0-31 (NC rounds 0,1)
//   A P2 = the rest                                             (KC 1,3 | NC 2,3)
//   B X  = rounds 0,1 (KC: columns 0-127; NC: k rows 0-31 -- both last read in phase 2 / 0)
//   B Y  = rounds 2,3
// Tile t+1's pieces go to the other stage (last read in tile t-1); B X of tile t+2 goes to
// this stage after its last B read (phase 2).  The DMA never drains to zero inside the loop:
// vmcnt(4) leaves two phases of pieces in flight, and each piece is issued >= 4 barrier
// intervals (>= 1,000 cycles) before the wait that retires it.
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

template <template <int, int, int> class LAT, template <int, int, int> class LBT, int EPI, bool STAMP = false>
__device__ __forceinline__ void mfma_gemm_256(const CoreParams& P) {
  constexpr int BM = 256, BN = 256, WN = 4, NT = 512;
  constexpr int FM = 8, FN = 4;
  constexpr int A_ELEMS = BM * BK, B_ELEMS = BN * BK;
  constexpr int STAGE = A_ELEMS + B_ELEMS;
  constexpr int SMEM = 2 * STAGE;
  static_assert(SMEM >= BM * EpiLayout<BN>::LD, "C staging must fit the two stages");
  constexpr int CPA = A_ELEMS / 8 / NT, CPB = B_ELEMS / 8 / NT;
  static_assert(CPA == 4 && CPB == 4, "pairs below assume 4 rounds per operand");
  using LA = LAT<BM, CPA, NT>;
  using LB = LBT<BN, CPB, NT>;
  constexpr bool A_KC = LA::KC, B_KC = LB::KC;
  static_assert(!loader_stateful<LA>::value && !loader_stateful<LB>::value, "rounds are issued out of order");
  // A pairs: KC -> {0,2} then {1,3}; NC -> {0,1} then {2,3}
  constexpr int AP1a = 0, AP1b = A_KC ? 2 : 1, AP2a = A_KC ? 1 : 2, AP2b = 3;
  __shared__ __attribute__((aligned(16))) short smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int grp = __builtin_amdgcn_readfirstlane(wave) >> 2;  // == wm, provably wave-uniform
  const int tiles_m = (P.M + BM - 1) / BM, tiles_n = (P.N + BN - 1) / BN;
  const BlkPos bp = blk_pos(P);
  int tm, tn;
  tile256_coords(bp.tile, tiles_m, tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = bp.split * P.k_per_split;
  int kend = kbeg + P.k_per_split;
  if (kend > P.K) kend = P.K;
  const int nk = (kend - kbeg + BK - 1) / BK;

  const LA la(P, true, m0, tid);
  const LB lb(P, false, n0, tid);
  const auto ra = loader_rsrc(la);
  const auto rb = loader_rsrc(lb);

  f4v acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  // one DMA round of an operand for K tile t into that tile's stage
  auto dma_a = [&](int t, auto ic) {
    constexpr int i = decltype(ic)::value;
    short* base = smem + (t & 1) * STAGE;
    CA_DMA_CHUNK(LA, la, ra, i, kbeg + t * BK, base + (i * NT + wave * 64) * 8);
  };
  auto dma_b = [&](int t, auto ic) {
    constexpr int i = decltype(ic)::value;
    short* base = smem + (t & 1) * STAGE + A_ELEMS;
    CA_DMA_CHUNK(LB, lb, rb, i, kbeg + t * BK, base + (i * NT + wave * 64) * 8);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  using IA1a = std::integral_constant<int, AP1a>;
  using IA1b = std::integral_constant<int, AP1b>;
  using IA2a = std::integral_constant<int, AP2a>;
  using IA2b = std::integral_constant<int, AP2b>;

  bf16x8 af[4], bfr[4];
  const int ar0 = wm * (BM / 2), bc0 = wn * (BN / WN);
  auto read_a = [&](const short* As, int mh, int kk) {
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = read_frag_sw<BM, A_KC>(As, ar0 + mh * 64 + i * 16, kk * 32, lane);
  };
  auto read_b = [&](const short* Bs, int kk) {
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[j] = read_frag_sw<BN, B_KC>(Bs, bc0 + j * 16, kk * 32, lane);
  };
  auto mma = [&](auto mhc) {
    constexpr int mh = decltype(mhc)::value;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[mh * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[mh * 4 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // diagnostic stamps (STAMP builds): for K tile nk/2, per segment the shader clock at its
  // start (after the opening barrier) and at its end (before the closing barrier), kept in
  // registers -- a store in the loop would disturb the counted vmcnt waits
  unsigned long long st[17];
  const int ts = nk / 2;
  auto stamp = [&](int t, auto kc) {
    if constexpr (STAMP) {
      if (t == ts) st[decltype(kc)::value] = __builtin_amdgcn_s_memtime();
    }
  };
  using S0 = std::integral_constant<int, 0>;  using S1 = std::integral_constant<int, 1>;
  using S2 = std::integral_constant<int, 2>;  using S3 = std::integral_constant<int, 3>;
  using S4 = std::integral_constant<int, 4>;  using S5 = std::integral_constant<int, 5>;
  using S6 = std::integral_constant<int, 6>;  using S7 = std::integral_constant<int, 7>;
  using S8 = std::integral_constant<int, 8>;  using S9 = std::integral_constant<int, 9>;
  using S10 = std::integral_constant<int, 10>;  using S11 = std::integral_constant<int, 11>;
  using S12 = std::integral_constant<int, 12>;  using S13 = std::integral_constant<int, 13>;
  using S14 = std::integral_constant<int, 14>;  using S15 = std::integral_constant<int, 15>;
  using S16 = std::integral_constant<int, 16>;

  // prologue: tile 0 in flight in full, then B pair X of tile 1; retire tile 0 minus A P2
  if (nk > 0) {
    dma_b(0, I0{});
    dma_b(0, I1{});
    dma_b(0, I2{});
    dma_b(0, I3{});
    dma_a(0, IA1a{});
    dma_a(0, IA1b{});
    dma_a(0, IA2a{});
    dma_a(0, IA2b{});
  }
  if (nk > 1) {
    dma_b(1, I0{});
    dma_b(1, I1{});
    vm_wait<4>();
  } else {
    vm_wait<2>();
  }
  bar256();
  if (grp == 1) bar256();

  for (int t = 0; t < nk; ++t) {
    const short* As = smem + (t & 1) * STAGE;
    const short* Bs = As + A_ELEMS;
    const bool n1 = t + 1 < nk, n2 = t + 2 < nk;
    // q0
    stamp(t, S0{});
    read_a(As, 0, 0);
    read_b(Bs, 0);
    if (n1) {
      dma_b(t + 1, I2{});
      dma_b(t + 1, I3{});
      vm_wait<4>();
    } else {
      vm_wait<0>();
    }
    lgkm_wait0();
    stamp(t, S1{});
    bar256();
    stamp(t, S2{});
    mma(I0{});
    stamp(t, S3{});
    bar256();
    // q1
    stamp(t, S4{});
    read_a(As, 1, 0);
    if (n1) {
      dma_a(t + 1, IA1a{});
      dma_a(t + 1, IA1b{});
    }
    lgkm_wait0();
    stamp(t, S5{});
    bar256();
    stamp(t, S6{});
    mma(I1{});
    stamp(t, S7{});
    bar256();
    // q2
    stamp(t, S8{});
    read_a(As, 0, 1);
    read_b(Bs, 1);
    if (n1) {
      dma_a(t + 1, IA2a{});
      dma_a(t + 1, IA2b{});
    }
    lgkm_wait0();
    stamp(t, S9{});
    bar256();
    stamp(t, S10{});
    mma(I0{});
    stamp(t, S11{});
    bar256();
    // q3
    stamp(t, S12{});
    read_a(As, 1, 1);
    if (n2) {
      dma_b(t + 2, I0{});
      dma_b(t + 2, I1{});
      vm_wait<4>();
    } else if (n1) {
      vm_wait<2>();
    } else {
      vm_wait<0>();
    }
    lgkm_wait0();
    stamp(t, S13{});
    bar256();
    stamp(t, S14{});
    mma(I1{});
    stamp(t, S15{});
    bar256();
    stamp(t, S16{});
  }
  if (grp == 0) bar256();
  if constexpr (STAMP) {
    if (lane == 0 && P.stamps) {
      unsigned long long* o = P.stamps + ((long)blockIdx.x * 8 + wave) * 17;
#pragma unroll
      for (int k = 0; k < 17; ++k) o[k] = st[k];
    }
  }
  __syncthreads();
  gemm_epilogue<BM, BN, 2, WN, EPI, SMEM>(P, acc, smem, m0, n0, tm, tid);
}

}  // namespace ca
