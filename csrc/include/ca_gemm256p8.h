// 256 x 256 x 64 MFMA GEMM core with a 4-phase-per-K-tile (8 phases per two K tiles)
// interleave over a double-buffered LDS-DMA image (gfx950 / CDNA4).
//
//   C[M,N] = sum_k A(m,k) * B(k,n)     bf16 operands, fp32 accumulation
//
// Geometry: one 512-thread workgroup per CU (2 waves per SIMD), K tile 64 deep.  The LDS
// holds two K tiles, each as four 16 KB half tiles: A top / bottom (128 rows x 64 k) and
// B left / right (128 columns x 64 k) -- 128 KB.  The C tile is four 128 x 128 quadrants;
// each PHASE computes one quadrant over one K tile with all 8 waves: waves 2 (M) x 4 (N),
// a 64 x 32 block per wave = 16 v_mfma_f32_16x16x32_bf16.  Quadrant order (0,0) (0,1)
// (1,1) (1,0) lets each phase read only ONE new half tile of fragments (A 8 or B 4
// ds_read_b128 per wave; the other operand's fragments stay in registers).
//
// Per phase: {fragment reads; one half tile of LDS-DMA (2 pieces per thread); [counted
// vmcnt]} barrier {lgkmcnt(0); 16 MFMAs at s_setprio 1} barrier.  Half tiles are restaged
// two phases after their last read and retired by ONE counted vmcnt(4) per K tile (two half
// tiles stay in flight; the loop never drains), read one phase after the wait:
//
//   K tile t, buffer b = t & 1      reads (buffer b)       DMA issued
//     q0 quadrant (0,0)              A top, B left          A bottom of t+1   (buffer b^1)
//     q1 quadrant (0,1)              B right                B left   of t+1   (buffer b^1)
//     q2 quadrant (1,1)              A bottom               A top    of t+2   (buffer b)
//     q3 quadrant (1,0)              B left                 B right  of t+2   (buffer b); vmcnt(4) -> t+1 complete
//
// Waves 4-7 run one barrier behind waves 0-3, so on every SIMD one wave multiplies while its
// partner reads LDS and issues DMA (MI355X_MICROARCH.md "Two waves per SIMD"); the two-phase
// restage distance keeps the write-after-read order safe under that stagger.  This is the
// structure of cdna_hip_programming.md section 5 "The 256^2 8-phase template" (measured there
// at ~1.33 PF/s at 4096^3 and ~1.47 PF/s at 8192^3 on random operands), written for this
// repo's loaders (GDenseKC / GDenseNC half tiles, XOR-swizzled lane-linear images) and its
// shared epilogue (QUAD fragment mapping).
#pragma once
#include "ca_gemm256.h"

namespace ca {

template <template <int, int, int> class LAT, template <int, int, int> class LBT, int EPI>
__device__ __forceinline__ void mfma_gemm_256p8(const CoreParams& P) {
  constexpr int BM = 256, BN = 256, NT = 512, HR = 128;
  constexpr int HT = HR * BK;  // shorts per half tile
  constexpr int SMEM = 8 * HT;  // 2 buffers x 4 half tiles = 128 KB
  static_assert(SMEM >= BM * EpiLayout<BN>::LD, "C staging must fit the operand image");
  using LA = LAT<HR, 2, NT>;
  using LB = LBT<HR, 2, NT>;
  static_assert(!loader_stateful<LA>::value && !loader_stateful<LB>::value, "stateless loaders only");
  constexpr bool A_KC = LA::KC, B_KC = LB::KC;
  constexpr int FM = 8, FN = 4;  // accumulator fragments per wave (2 x 2 quadrants of 4 x 2)
  __shared__ __attribute__((aligned(16))) short smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / 4, wn = wave % 4;
  const int grp = __builtin_amdgcn_readfirstlane(wave) >> 2;
  const int tiles_m = (P.M + BM - 1) / BM, tiles_n = (P.N + BN - 1) / BN;
  const BlkPos bp = blk_pos(P);
  int tm, tn;
  tile256_coords(bp.tile, tiles_m, tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = bp.split * P.k_per_split;
  int kend = kbeg + P.k_per_split;
  if (kend > P.K) kend = P.K;
  const int nk = (kend - kbeg + BK - 1) / BK;

  const LA la0(P, true, m0, tid), la1(P, true, m0 + HR, tid);
  const LB lb0(P, false, n0, tid), lb1(P, false, n0 + HR, tid);
  const auto ra0 = loader_rsrc(la0), ra1 = loader_rsrc(la1);
  const auto rb0 = loader_rsrc(lb0), rb1 = loader_rsrc(lb1);

  // half tile h of buffer b: 0 A top, 1 A bottom, 2 B left, 3 B right
  auto region = [&](int b, int h) { return smem + (b * 4 + h) * HT; };
  auto dma = [&](int t, int h) {
    const int k0 = kbeg + t * BK;
    short* dst = region(t & 1, h);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      short* d = dst + (i * NT + wave * 64) * 8;
      if (h == 0) CA_DMA_CHUNK(LA, la0, ra0, i, k0, d);
      else if (h == 1) CA_DMA_CHUNK(LA, la1, ra1, i, k0, d);
      else if (h == 2) CA_DMA_CHUNK(LB, lb0, rb0, i, k0, d);
      else CA_DMA_CHUNK(LB, lb1, rb1, i, k0, d);
    }
  };

  f4v acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  bf16x8 af[4][2], bfr[2][2];  // this phase's fragments: A 4 rows x 2 k halves, B 2 cols x 2 k halves
  auto read_a = [&](const short* half) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) af[i][kk] = read_frag_sw<HR, A_KC>(half, wm * 64 + i * 16, kk * 32, lane);
  };
  auto read_b = [&](const short* half) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) bfr[j][kk] = read_frag_sw<HR, B_KC>(half, wn * 32 + j * 16, kk * 32, lane);
  };
  auto mfma_q = [&](int qm, int qn) {
    lgkm_wait0();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[qm * 4 + i][qn * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j][kk], af[i][kk], acc[qm * 4 + i][qn * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // prologue: all of K tile 0, and the half tiles of tile 1 that K tile -1 would have issued
  if (nk > 0) {
    dma(0, 0);
    dma(0, 3);
    dma(0, 1);
    dma(0, 2);
  }
  if (nk > 1) {
    dma(1, 0);
    dma(1, 3);
    vm_wait<4>();
  } else {
    vm_wait<0>();
  }
  bar256();
  if (grp == 1) bar256();

  for (int t = 0; t < nk; ++t) {
    const int b = t & 1;
    // q0: quadrant (0,0)
    read_a(region(b, 0));
    read_b(region(b, 2));
    if (t + 1 < nk) dma(t + 1, 1);
    bar256();
    mfma_q(0, 0);
    bar256();
    // q1: quadrant (0,1)
    read_b(region(b, 3));
    if (t + 1 < nk) dma(t + 1, 2);
    bar256();
    mfma_q(0, 1);
    bar256();
    // q2: quadrant (1,1)
    read_a(region(b, 1));
    if (t + 2 < nk) dma(t + 2, 0);
    bar256();
    mfma_q(1, 1);
    bar256();
    // q3: quadrant (1,0); K tile t+1 must be complete before the next q0 reads it
    read_b(region(b, 2));
    if (t + 2 < nk) {
      dma(t + 2, 3);
      vm_wait<4>();
    } else {
      vm_wait<0>();
    }
    bar256();
    mfma_q(1, 0);
    bar256();
  }
  if (grp == 0) bar256();
  __syncthreads();
  gemm_epilogue<BM, BN, 2, 4, EPI, SMEM, 1, FM, FN, true>(P, acc, smem, m0, n0, tm, tid);
}

}  // namespace ca
