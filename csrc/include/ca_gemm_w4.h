// 256 x BN x 64 MFMA GEMM core, FOUR waves, one workgroup per CU, accumulators pinned to the
// accumulator register file (gfx950 / CDNA4).
//
//   C[M,N] = sum_k A(m,k) * B(k,n)     bf16 operands, fp32 accumulation
//
// The structure the vendor library runs on these shapes (one wave per SIMD, every wave
// multiplying a 128 x BN/2 block all the time, one barrier per K tile), which HIP C++ could not
// express in round 5: with 256 / 192 / 160 accumulator registers per lane the compiler kept
// shuffling the MFMA results between the VGPR and AGPR halves of the register file (~220-450
// v_accvgpr moves per K tile, docs/performance.md "A 4-wave, one-barrier GEMM core").  Here every
// MFMA is an inline-asm statement whose accumulator operand is constrained to AGPRs ("+a"): the
// accumulators are written once (bias / zero), live in a[0:4*FM*FN-1] for the whole K loop and
// are read once by the epilogue; the A / B fragments stay compiler-scheduled ds_reads into
// VGPRs, so hipcc still interleaves the next fragments' reads with the MFMAs and counts lgkmcnt.
//
// Hazards the compiler does not see through an asm statement (cdna_hip_programming.md §5.7):
//   * MFMA operands come straight from ds_read_b128 / ds_read_b64_tr_b16 (no VALU writes them);
//   * consecutive MFMAs on one accumulator form an accumulate chain (no wait states);
//   * after the K loop one `s_nop` block separates the last MFMA from the epilogue's
//     v_accvgpr_read, and every accumulator passes through an empty asm statement ordered
//     after it, so no read is scheduled above the wait.
//
// K loop (two LDS stages, LDS-DMA with the source-side XOR swizzle of the glds core):
//     wait vmcnt(0) [tile t landed] ; lgkmcnt(0) ; s_barrier [every wave done with t-1]
//     DMA tile t+1 into the other stage ; fragments + MFMAs of tile t
// The DMA of tile t+1 is in flight for the whole of tile t's MFMAs (128 x BN/2 x 64 per wave:
// 8 x FN x 2 MFMAs), so one stage ahead hides it; raw s_barrier, never __syncthreads (whose
// fence would drain the DMA).
#pragma once
#include "ca_mfma_core.h"

namespace ca {

// acc += B-fragment x A-fragment (the operand order of mfma_acc: C^T tile, four consecutive
// columns of one row per lane), accumulator in AGPRs
__device__ __forceinline__ void mfma_agpr(f4v& acc, const bf16x8& b, const bf16x8& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}

// DIAG (bench builds only): 1 = no DMA after the prologue (MFMA + LDS-read ceiling, wrong
// results); 2 = no MFMAs (load-path floor, wrong results)
template <int BN, template <int, int, int> class LAT, template <int, int, int> class LBT, int EPI, int DIAG = 0>
__device__ __forceinline__ void mfma_gemm_w4(const CoreParams& P) {
  constexpr int BM = 256, NT = 256, WM = 2, WN = 2;
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;
  static_assert(BN % 32 == 0, "BN: 32-column steps (2 waves x 16-column fragments)");
  constexpr int A_ELEMS = BM * BK, B_ELEMS = BN * BK;
  constexpr int STAGE = A_ELEMS + B_ELEMS;
  constexpr int EPI_LD = EpiLayout<BN>::LD;
  constexpr int SMEM = (2 * STAGE > BM * EPI_LD ? 2 * STAGE : BM * EPI_LD);
  constexpr int CPA = A_ELEMS / 8 / NT, CPB = B_ELEMS / 8 / NT;
  static_assert(A_ELEMS % (8 * NT) == 0 && B_ELEMS % (8 * NT) == 0, "tile chunks must divide threads");
  static_assert(SMEM * 2 <= 160 * 1024, "LDS");
  using LA = LAT<BM, CPA, NT>;
  using LB = LBT<BN, CPB, NT>;
  constexpr bool A_KC = LA::KC, B_KC = LB::KC;
  __shared__ __attribute__((aligned(16))) short smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_m = (P.M + BM - 1) / BM, tiles_n = (P.N + BN - 1) / BN;
  (void)tiles_m;
  const BlkPos bp = blk_pos(P);
  const int tm = bp.tile / tiles_n, tn = bp.tile % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = bp.split * P.k_per_split;
  int kend = kbeg + P.k_per_split;
  if (kend > P.K) kend = P.K;
  const int nk = (kend - kbeg + BK - 1) / BK;

  LA la(P, true, m0, tid);
  LB lb(P, false, n0, tid);
  const auto ra = loader_rsrc(la);
  const auto rb = loader_rsrc(lb);
  // wave-uniform LDS destination of this wave's piece q of a stage (SGPR arithmetic: M0 is
  // written from a scalar, no v_readfirstlane per piece)
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  constexpr int NPC = CPA + CPB;  // DMA pieces per thread per K tile
  auto dma_piece = [&](int q, int k1, short* base) {
    if (q < CPA) CA_DMA_CHUNK(LA, la, ra, q, k1, base + (q * NT + wv * 64) * 8);
    else CA_DMA_CHUNK(LB, lb, rb, q - CPA, k1, base + A_ELEMS + ((q - CPA) * NT + wv * 64) * 8);
  };

  f4v acc[FM][FN];
  constexpr bool BIAS0 = EPI == EPI_BF16;
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

  // One K tile, software-pipelined by hand (the MFMA statements are volatile, so program
  // order is issue order): 2 FM steps of FN MFMAs (one A row of fragments each); step s reads
  // the A fragment of step s+1, the first FN steps also read the next K half's B fragments,
  // and the NPC DMA pieces of tile t+1 are spread over the steps -- every LDS read and DMA
  // issue sits in the shadow of the MFMAs before it.
  auto tile = [&](int t) {
    const short* As = smem + (t & 1) * STAGE;
    const short* Bs = As + A_ELEMS;
    short* nb = smem + ((t + 1) & 1) * STAGE;
    const bool pf = t + 1 < nk;
    const int k1 = kbeg + (t + 1) * BK;
    bf16x8 b0[FN], b1[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) b0[j] = read_frag_sw<BN, B_KC>(Bs, wn * (BN / WN) + j * 16, 0, lane);
    bf16x8 acur = read_frag_sw<BM, A_KC>(As, wm * (BM / WM), 0, lane);
    constexpr int NS = 2 * FM;
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      const int i = st % FM, kk = st / FM;
      bf16x8 anxt = acur;
      if (st + 1 < NS) anxt = read_frag_sw<BM, A_KC>(As, wm * (BM / WM) + ((st + 1) % FM) * 16, ((st + 1) / FM) * 32, lane);
      if (kk == 0 && i < FN) b1[i] = read_frag_sw<BN, B_KC>(Bs, wn * (BN / WN) + i * 16, 32, lane);
      if (pf && DIAG != 1) {
#pragma unroll
        for (int q = (st * NPC) / NS; q < ((st + 1) * NPC) / NS; ++q) dma_piece(q, k1, nb);
      }
      if constexpr (DIAG != 2) {
#pragma unroll
        for (int j = 0; j < FN; ++j) mfma_agpr(acc[i][j], kk == 0 ? b0[j] : b1[j], acur);
      } else {
#pragma unroll
        for (int j = 0; j < FN; ++j) asm volatile("" ::"v"(b0[j]), "v"(b1[j]), "v"(acur));
      }
      acur = anxt;
    }
    if constexpr (loader_stateful<LA>::value) la.advance();
    if constexpr (loader_stateful<LB>::value) lb.advance();
  };

  if (nk > 0) {
#pragma unroll
    for (int q = 0; q < NPC; ++q) dma_piece(q, kbeg, smem);
  }
  for (int t = 0; t < nk; ++t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    tile(t);
  }
  // the last MFMA's result before any other reader (16x16x32 bf16: 8 passes -> 12 wait states),
  // then every accumulator through an asm statement ordered after the wait
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) asm volatile("" : "+a"(acc[i][j]));
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // every wave done reading the operand stages (the epilogue reuses the LDS)
  gemm_epilogue<BM, BN, WM, WN, EPI, SMEM, 1, FM, FN, false, BIAS0>(P, acc, smem, m0, n0, tm, tid);
}

}  // namespace ca
