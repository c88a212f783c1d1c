// Persistent resident-weight GEMM for the small-K, memory-bound NT GEMMs of ResNet's 1x1
// forward convolutions (gfx950 / CDNA4):
//
//   C[M, N] = A[M, K] * B[N, K]^T      K, N <= 256, B * K <= 32K elements, M in the millions
//
// With K = 64..256 a 128 x N output tile is one to four K steps: the data-parallel 128 x 128
// core spends most of each block on its prologue (first DMA round trip), its epilogue (C
// through LDS, BN statistics) and block turnover, and re-reads B once per tile.  Here one
// 512-thread workgroup per CU (two per CU when the LDS allows) owns a contiguous range of
// 128-row tiles and
//   * keeps the whole B (the conv weights, N x K) resident in LDS, loaded once;
//   * streams the A tiles through an NS-deep LDS-DMA ring (buffer_load ... lds), issued
//     NS - 1 K steps ahead, so the next tiles' loads are in flight during this tile's MFMAs
//     AND its epilogue stores;
//   * retires each step with a COUNTED vmcnt: loads, LDS-DMA and stores count together in
//     issue order (MI355X_MICROARCH.md, constants), every thread issues exactly the same
//     sequence (buffer stores, rows past M dropped by the range check rather than skipped),
//     so the number of younger operations at each wait is known -- the loop never drains;
//   * accumulates the BN-forward statistics [sum | sum of squares] of the stored bf16
//     values in registers across ALL its tiles and writes ONE partial row per workgroup
//     (gridDim.x rows instead of M / 128: 256 instead of 25,088 at ResNet-50 stage 1, b1024).
//
// Column chunks (P.prw_chunks = NCH > 1): a weight too large for LDS (ResNet's conv3
// expansions, N = 512..2048 at K = 128..512) is split into NCH chunks of BN columns; NCH
// workgroups share one row range, each with its chunk of B resident, and stream the SAME A
// tiles.  The NCH workgroups of a range are dealt to one XCD (block b runs on XCD b % 8), start
// together and run the same step sequence, so an A tile is fetched from HBM once and read by the
// other NCH - 1 from that XCD's L2 or the MALL (measured: spreading the chunks over the XCDs
// costs ~1 %, so the re-reads are not the bound).  The data-parallel 128 x 128 core ran these
// write-heavy shapes at 2.4-3.1 TB/s; this runs ResNet-50's stage-2 conv3 ~15 % faster (3.7
// TB/s), stage 3 ~4 % (gemm.hip prw_kind).  Partials: one row per range, each chunk writing its
// BN columns.
// Barriers are bare s_barrier (a __syncthreads fence would wait for vmcnt(0) and drain the
// prefetch); LDS writes are ordered by lgkmcnt(0) before them.
#pragma once
#include "ca_gemm256.h"

namespace ca {

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (the instruction takes an immediate);
// n beyond the table waits for everything -- correct, only slower.
__device__ __forceinline__ void vm_wait_rt(int n) {
#define CA_VW(k) \
  case k:        \
    vm_wait<k>(); \
    break;
  switch (n) {
    CA_VW(1) CA_VW(2) CA_VW(3) CA_VW(4) CA_VW(5) CA_VW(6) CA_VW(7) CA_VW(8) CA_VW(9) CA_VW(10) CA_VW(11)
    CA_VW(12) CA_VW(13) CA_VW(14) CA_VW(15) CA_VW(16) CA_VW(17) CA_VW(18) CA_VW(19) CA_VW(20) CA_VW(21)
    CA_VW(22) CA_VW(23) CA_VW(24) CA_VW(25) CA_VW(26) CA_VW(27) CA_VW(28) CA_VW(29) CA_VW(30) CA_VW(31)
    CA_VW(32) CA_VW(33) CA_VW(34) CA_VW(35) CA_VW(36) CA_VW(37) CA_VW(38) CA_VW(39) CA_VW(40)
    default:
      vm_wait<0>();
  }
#undef CA_VW
}

template <int BN, int KT, int NS>
struct PrwGeom {
  static constexpr int NT = 512, BM = 128, WM = 2, WN = 4;
  static constexpr int NK = KT / 64;
  static constexpr int A_ST = BM * 64;            // shorts per A stage
  static constexpr int B_ELEMS = BN * KT;         // resident B (NK slices of [BN][64])
  static constexpr int C_ELEMS = BM * EpiLayout<BN>::LD;
  static constexpr int SHORTS = B_ELEMS + NS * A_ST + C_ELEMS;
  static constexpr int BYTES = SHORTS * 2;
};

template <int BN, int KT, int NS, bool STATS>
__device__ __forceinline__ void prw_gemm_body(const CoreParams& P) {
  using G = PrwGeom<BN, KT, NS>;
  constexpr int NT = G::NT, BM = G::BM, WN = G::WN, NK = G::NK, A_ST = G::A_ST;
  constexpr int FM = BM / G::WM / 16, FN = BN / WN / 16;
  constexpr int CPA = A_ST / 8 / NT;      // A chunks (16 B) per thread and K step
  constexpr int CPB = BN * 64 / 8 / NT;   // B chunks per thread and K slice
  constexpr int CG = BN / 8, RP = NT / CG, IT = BM / RP;  // epilogue: column groups, row parts, rows/thread
  static_assert(KT % 64 == 0 && NK >= 1 && CPA >= 1 && CPB >= 1 && FN >= 1 && NS >= 2, "geometry");
  static_assert(NT % CG == 0 && BM % RP == 0, "epilogue geometry");
  static_assert(2 * RP * BN * 4 <= NS * A_ST * 2, "statistics rows must fit the A ring");
  using EL = EpiLayout<BN>;
  __shared__ __attribute__((aligned(16))) short smem[G::SHORTS];
  short* const Bs = smem;
  short* const As = smem + G::B_ELEMS;
  short* const Cs = As + NS * A_ST;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int T = (P.M + BM - 1) / BM;
  // (row range, column chunk) of this workgroup; with chunks the host makes gridDim.x a
  // multiple of 8 * NCH, and the chunks of a range share the XCD b % 8
  const int NCH = P.prw_chunks > 1 ? P.prw_chunks : 1;
  int range = blockIdx.x, chunk = 0, R = gridDim.x;
  if (NCH > 1) {
    const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
    const int rpx = (gridDim.x >> 3) / NCH;  // ranges per XCD
    range = xcd * rpx + j / NCH;
    chunk = j % NCH;
    R = gridDim.x / NCH;
  }
  const int t0 = (int)((long)range * T / R), t1 = (int)((long)(range + 1) * T / R);
  const int nsteps = (t1 - t0) * NK;
  const long col0 = (long)chunk * BN;  // first output column (and B row) of this chunk
  const long ntot = (long)NCH * BN;    // == P.N

  // A chunk i of this thread: tile row (tid >> 3) + 64 i, swizzled 16-B slot (tid & 7) ^ (row & 7)
  const int arow = tid >> 3;
  const int acol = ((tid & 7) ^ (arow & 7)) << 3;
  const uint32_t avoff = (uint32_t)((arow * P.lda + acol) * 2);
  const uint32_t astep = (uint32_t)(NT / 8) * (uint32_t)P.lda * 2u;

  int issued = 0;   // vector-memory operations this thread has issued (uniform over threads)
  int mk[NS - 1];   // `issued` right after each outstanding A step's DMA, oldest first
#pragma unroll
  for (int q = 0; q < NS - 1; ++q) mk[q] = 0;

  // resident B: NK slices [BN][64], same swizzle as the A stages
  {
    const auto rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(P.B + col0 * P.ldb), (short)0,
                                                      (int)buf_span((long)BN * P.ldb * 2), 0x00020000);
#pragma unroll
    for (int kk = 0; kk < NK; ++kk)
#pragma unroll
      for (int i = 0; i < CPB; ++i) {
        const int c = tid + i * NT, row = c >> 3, lc = (c & 7) ^ (row & 7);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(Bs + kk * BN * 64 + (i * NT + wave * 64) * 8), 16,
                                                 (row * (int)P.ldb + kk * 64 + lc * 8) * 2, 0, 0, 0);
      }
    issued += NK * CPB;
  }
  auto issue_a = [&](int q) {
    const int tile = t0 + q / NK, kk = q % NK;
    const long r0 = (long)tile * BM;
    const auto ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(P.A + r0 * P.lda), (short)0,
                                                      (int)buf_span((P.M - r0) * P.lda * 2), 0x00020000);
    short* dst = As + (q % NS) * A_ST;
#pragma unroll
    for (int i = 0; i < CPA; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(dst + (i * NT + wave * 64) * 8), 16,
                                               avoff + (uint32_t)i * astep + (uint32_t)kk * 128u, 0, 0, 0);
    issued += CPA;
  };
#pragma unroll
  for (int q = 0; q < NS - 1; ++q) {
    if (q < nsteps) issue_a(q);
    mk[q] = issued;
  }

  f4v acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  float ssum[8], ssq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) ssum[j] = ssq[j] = 0.f;
  const int ecol = (tid % CG) * 8, epart = tid / CG;
  const int rbase = wm * (BM / G::WM) + (lane & 15), cbase = wn * (BN / WN) + 4 * (lane >> 4);

  for (int s = 0; s < nsteps; ++s) {
    vm_wait_rt(issued - mk[0]);  // this thread's pieces of step s (and B) have landed
    bar256();                    // ... everyone's; and every wave is done with step s - 1's stage
#pragma unroll
    for (int q = 0; q < NS - 2; ++q) mk[q] = mk[q + 1];
    if (s + NS - 1 < nsteps) issue_a(s + NS - 1);  // refills the stage step s - 1 read
    mk[NS - 2] = issued;
    const int kk = s % NK;
    const short* Ast = As + (s % NS) * A_ST;
    const short* Bsl = Bs + kk * BN * 64;
#pragma unroll
    for (int kq = 0; kq < 64; kq += 32) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = read_frag_sw<BM, true>(Ast, wm * (BM / G::WM) + i * 16, kq, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = read_frag_sw<BN, true>(Bsl, wn * (BN / WN) + j * 16, kq, lane);
      mfma_acc<FM, FN>(acc, af, bfr);
    }
    if (kk != NK - 1) continue;

    // ---- epilogue of tile t: acc -> LDS (bf16) -> 16-B buffer stores, statistics in registers
    const long m0 = (long)(t0 + s / NK) * BM;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        s4v pk;
#pragma unroll
        for (int r = 0; r < 4; ++r) pk[r] = (short)f2bf(acc[i][j][r]);
        *reinterpret_cast<s4v*>(Cs + EL::idx(rbase + i * 16, cbase + j * 16)) = pk;
        acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
      }
    lgkm_wait0();
    bar256();
    const auto rc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<bf16_t*>(P.C) + m0 * P.ldc + col0, (short)0,
                                                      (int)buf_span((P.M - m0) * P.ldc * 2 - col0 * 2), 0x00020000);
    s8v v[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) v[it] = *reinterpret_cast<const s8v*>(Cs + EL::idx(epart + it * RP, ecol));
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[it]), rc,
                                             (int)(((epart + it * RP) * P.ldc + ecol) * 2), 0, 0);
      if constexpr (STATS) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float a = bf2f((bf16_t)v[it][j]);
          ssum[j] += a;
          ssq[j] += a * a;
        }
      }
    }
    issued += IT;
  }
  vm_wait<0>();
  if constexpr (STATS) {
    // [sum | sum of squares] per column over this workgroup's tiles: registers -> LDS (the
    // A ring, idle now) -> one thread per column -> partial row blockIdx.x
    lgkm_wait0();
    bar256();
    float* sred = reinterpret_cast<float*>(As);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sred[epart * BN + ecol + j] = ssum[j];
      sred[(RP + epart) * BN + ecol + j] = ssq[j];
    }
    lgkm_wait0();
    bar256();
    for (int c = tid; c < BN; c += NT) {
      float ts = 0.f, tq = 0.f;
      for (int pp = 0; pp < RP; ++pp) {
        ts += sred[pp * BN + c];
        tq += sred[(RP + pp) * BN + c];
      }
      float* st = P.stats + (long)range * 2 * ntot + col0;
      st[c] = ts;
      st[ntot + c] = tq;
    }
  }
}

}  // namespace ca
