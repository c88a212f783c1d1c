// 256 x 256 x 64 MFMA GEMM core over a double-buffered LDS-DMA image, two staggered wave
// groups, counted vmcnt (gfx950 / CDNA4).
//
//   C[M,N] = sum_k A(m,k) * B(k,n)     bf16 operands, fp32 accumulation
//
// Geometry: one 512-thread workgroup per CU (2 waves per SIMD), K tile 64 deep.  The LDS
// holds two K tiles, each as four 16 KB half tiles: A top / bottom (128 rows x 64 k) and
// B left / right (128 columns x 64 k) -- 128 KB.  Waves are 2 (M) x 4 (N); every phase is
// {fragment reads; s_waitcnt lgkmcnt(0); LDS-DMA of restaged half tiles (2 pieces per thread
// each); counted vmcnt} barrier {MFMAs at s_setprio 1} barrier, and waves 4-7 run one barrier
// behind waves 0-3, so on every SIMD one wave multiplies while its partner reads LDS and
// issues DMA (MI355X_MICROARCH.md "Two waves per SIMD").  Because each phase retires its own
// LDS reads before its first barrier, a half tile is restaged ONE phase after its last read;
// a half tile's data is waited for (counted vmcnt) before the first barrier of a phase that
// precedes the phase reading it (cdna_hip_programming.md section 5, RAW / WAR rules with the
// stagger).  The loop never drains vmcnt to 0.
//
// PHASES = 2 (default): one C HALF per phase, 32 MFMAs per wave between barriers.
//   K tile t, buffer b = t & 1     reads (buffer b)                 DMA issued
//     P1 top half    (qm 0)        A top, B left, B right           A bottom of t+1 (buffer b^1)
//     P2 bottom half (qm 1)        A bottom (B held in registers)   A top, B left, B right of t+2
//                                                                   (buffer b); vmcnt(6) -> t+1 complete
// PHASES = 4: one C QUADRANT per phase, 16 MFMAs per wave between barriers (the layout of
//   cdna_hip_programming.md "The 256^2 8-phase template"): quadrant order (0,0) (0,1) (1,1)
//   (1,0), one new half tile of fragments per phase, A bottom / B left of t+1 and A top /
//   B right of t+2 restaged two phases after their last reads, vmcnt(4) once per K tile.
//
// Measured on MI355X, one process, random operands (bin/gemm_bench, profiles/r4_gemm/):
// PHASES 2 reaches 1,178-1,228 TF/s at 4096^3 and 1,245-1,260 at 8192^3 (MFMA busy 0.70),
// PHASES 4 1,050-1,110 / 1,168-1,190 (busy 0.61), the ring core of ca_gemm256.h 1,097-1,158 /
// 1,172-1,183 (busy 0.65).  Variants that waited for each half tile one phase before it is
// read (four half tiles in flight) or rotated A bottom over three slots (144 KB) gave the
// half-tile loads more latency budget and were NOT faster: the barrier count per MFMA, not the
// load latency, is what the extra MFMAs per phase buy back.  Epilogue: the shared
// gemm_epilogue with the quadrant fragment mapping (QUAD).
#pragma once
#include "ca_gemm256.h"

namespace ca {

// The two-phase K loop for ONE 256 x 256 tile at (m0, n0) over K elements [kbeg, kend), into
// `acc` (zeroed here), on the 128-KB operand image `smem`.  Returns with both wave groups
// re-aligned and every LDS read retired (__syncthreads): the caller may reuse the LDS.  Used
// by the data-parallel kernel below (one tile per workgroup) and by the stream-K kernel
// (mfma_gemm_256p8_sk: several tile segments per workgroup).
template <template <int, int, int> class LAT, template <int, int, int> class LBT>
struct P8Loop {
__device__ static __forceinline__ void run(const CoreParams& P, int m0, int n0, int kbeg, int kend, short* smem,
                                           f4v (&acc)[8][4]) {
  constexpr int NT = 512, HR = 128;
  constexpr int HT = HR * BK;  // shorts per half tile
  using LA = LAT<HR, 2, NT>;
  using LB = LBT<HR, 2, NT>;
  static_assert(!loader_stateful<LA>::value && !loader_stateful<LB>::value, "stateless loaders only");
  constexpr bool A_KC = LA::KC, B_KC = LB::KC;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / 4, wn = wave % 4;
  const int grp = __builtin_amdgcn_readfirstlane(wave) >> 2;
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
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
  // fragments: A 4 rows x 2 k halves of one A half tile; B 2 cols x 2 k halves of the left
  // (bfl) and right (bfr) B half tiles
  bf16x8 af[4][2], bfl[2][2], bfr[2][2];
  auto read_a = [&](const short* half) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) af[i][kk] = read_frag_sw<HR, A_KC>(half, wm * 64 + i * 16, kk * 32, lane);
  };
  auto read_b = [&](bf16x8 (&f)[2][2], const short* half) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) f[j][kk] = read_frag_sw<HR, B_KC>(half, wn * 32 + j * 16, kk * 32, lane);
  };
  // C half qm (quadrants (qm,0), (qm,1)) from af, bfl and bfr: 32 MFMAs
  auto mfma_h = [&](int qm) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[qm * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(j < 2 ? bfl[j][kk] : bfr[j - 2][kk], af[i][kk],
                                                                       acc[qm * 4 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // prologue: K tile 0, and tile 1's A top / B left / B right (what "P2 of tile -1" issues)
  if (nk > 0) {
    dma(0, 0);
    dma(0, 2);
    dma(0, 3);
    dma(0, 1);
  }
  if (nk > 1) {
    dma(1, 0);
    dma(1, 2);
    dma(1, 3);
    vm_wait<6>();
  } else {
    vm_wait<0>();
  }
  bar256();
  if (grp == 1) bar256();
  for (int t = 0; t < nk; ++t) {
    const int b = t & 1;
    // P1: top C half
    read_a(region(b, 0));
    read_b(bfl, region(b, 2));
    read_b(bfr, region(b, 3));
    lgkm_wait0();
    if (t + 1 < nk) dma(t + 1, 1);
    bar256();
    mfma_h(0);
    bar256();
    // P2: bottom C half; K tile t+1 must be complete before the next P1 reads it
    read_a(region(b, 1));
    lgkm_wait0();
    if (t + 2 < nk) {
      dma(t + 2, 0);
      dma(t + 2, 2);
      dma(t + 2, 3);
      vm_wait<6>();
    } else {
      vm_wait<0>();
    }
    bar256();
    mfma_h(1);
    bar256();
  }
  if (grp == 0) bar256();
  __syncthreads();
}
};

template <template <int, int, int> class LAT, template <int, int, int> class LBT, int EPI, int PHASES = 2>
__device__ __forceinline__ void mfma_gemm_256p8(const CoreParams& P) {
  static_assert(PHASES == 2 || PHASES == 4, "2 or 4 phases per K tile");
  constexpr int BM = 256, BN = 256, NT = 512, HR = 128;
  constexpr int HT = HR * BK;   // shorts per half tile
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

  // fragments: A 4 rows x 2 k halves of one A half tile; B 2 cols x 2 k halves of the left
  // (bfl) and right (bfr) B half tiles (PHASES 4 uses bfl only)
  bf16x8 af[4][2], bfl[2][2], bfr[2][2];
  auto read_a = [&](const short* half) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) af[i][kk] = read_frag_sw<HR, A_KC>(half, wm * 64 + i * 16, kk * 32, lane);
  };
  auto read_b = [&](bf16x8 (&f)[2][2], const short* half) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) f[j][kk] = read_frag_sw<HR, B_KC>(half, wn * 32 + j * 16, kk * 32, lane);
  };
  // C quadrant (qm, qn) from af and bfl: 16 MFMAs
  auto mfma_q = [&](int qm, int qn) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[qm * 4 + i][qn * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfl[j][kk], af[i][kk], acc[qm * 4 + i][qn * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // C half qm (quadrants (qm,0), (qm,1)) from af, bfl and bfr: 32 MFMAs
  auto mfma_h = [&](int qm) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[qm * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(j < 2 ? bfl[j][kk] : bfr[j - 2][kk], af[i][kk],
                                                                       acc[qm * 4 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  if constexpr (PHASES == 2) {
    P8Loop<LAT, LBT>::run(P, m0, n0, kbeg, kend, smem, acc);
    gemm_epilogue<BM, BN, 2, 4, EPI, SMEM, 1, FM, FN, true>(P, acc, smem, m0, n0, tm, tid);
    return;
  } else {
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
      read_b(bfl, region(b, 2));
      if (t + 1 < nk) dma(t + 1, 1);
      bar256();
      lgkm_wait0();
      mfma_q(0, 0);
      bar256();
      // q1: quadrant (0,1)
      read_b(bfl, region(b, 3));
      if (t + 1 < nk) dma(t + 1, 2);
      bar256();
      lgkm_wait0();
      mfma_q(0, 1);
      bar256();
      // q2: quadrant (1,1)
      read_a(region(b, 1));
      if (t + 2 < nk) dma(t + 2, 0);
      bar256();
      lgkm_wait0();
      mfma_q(1, 1);
      bar256();
      // q3: quadrant (1,0); K tile t+1 must be complete before the next q0 reads it
      read_b(bfl, region(b, 2));
      if (t + 2 < nk) {
        dma(t + 2, 3);
        vm_wait<4>();
      } else {
        vm_wait<0>();
      }
      bar256();
      lgkm_wait0();
      mfma_q(1, 0);
      bar256();
    }
  }
  if (grp == 0) bar256();
  __syncthreads();
  gemm_epilogue<BM, BN, 2, 4, EPI, SMEM, 1, FM, FN, true>(P, acc, smem, m0, n0, tm, tid);
}

// ---------------------------------------------------------------------------------------
// Stream-K over the two-phase core, for GEMMs whose 256 x 256 grid is less than a few rounds
// of the chip (BERT-base at M = 8192: QKV 288 tiles, FFN1 forward / FFN2 input gradient 384,
// FFN2 forward / FFN1 and QKV input gradients 96, attention output 96 -- 1.1-1.5 rounds or
// less, which left up to half the CUs idle in the last round and sent these shapes to the 128
// core, with twice the L2 -> LDS traffic per MFMA).
//
// The (tile, K iteration) space -- tiles x ipt iterations of BK = 64 -- is cut into gridDim.x
// equal contiguous ranges, one per workgroup (one 128-KB workgroup per CU).  Ranges are dealt
// to XCDs contiguously (xcd_remap), tiles in the 256-core's grouped order, so the workgroups
// that share a tile's K range are neighbours on one XCD.  A workgroup runs its range as
// segments of P8Loop::run; a tile covered by one segment goes straight to the epilogue.  A split
// tile has a static OWNER: the workgroup whose segment holds the tile's first K iteration
// (the last segment of its range, so it is normally the last to reach the tile).  Every other
// contributor stores its fp32 partial tile (16-B stores, [32 fragments][512 threads]) and
// publishes it with the agent-scope release recipe of cdna_hip_programming.md section 5 (all
// waves retire their stores, barrier, one lane: release fence, wait, relaxed agent-scope
// atomic add on the tile's ticket).  The owner polls the ticket (relaxed agent-scope loads)
// until every contributor arrived, acquires, adds the partials in contributor order to its own
// accumulator (a fixed order: the result does not depend on timing), resets the ticket for the
// next launch and runs the ordinary epilogue (bias / activation / pre-activation / act').
// No contributor ever waits except an owner, and every contributor it waits for has already
// finished its MFMAs or is running: the grid is gridDim.x <= CU count single-workgroup CUs.
struct SkParams {
  float* part;    // [gridDim.x][256 * 256] partial tiles, slot w = range w's first segment
  int* ticket;    // [tiles] arrival counts, zero between launches (the owner resets its tile's);
                  // ticket[err_index] = 1 if an owner's bounded wait ever ran out
  int ipt;        // K iterations per tile
  int err_index;
  int total;      // tiles * ipt (< 2^31 / CU count: host-checked)
};

// 32-bit range arithmetic (the scalar registers are as scarce as the vector ones here)
__device__ __forceinline__ int sk_start(int w, int total, int G) {
  return (int)(((unsigned long long)(unsigned)w * (unsigned)total) / (unsigned)G);
}

// the range index whose [start, next start) holds iteration x
__device__ __forceinline__ int sk_owner_of(int x, int total, int G) {
  int w = (int)(((unsigned long long)(unsigned)x * (unsigned)G) / (unsigned)total);
  while (w + 1 < G && sk_start(w + 1, total, G) <= x) ++w;
  while (w > 0 && sk_start(w, total, G) > x) --w;
  return w;
}

template <template <int, int, int> class LAT, template <int, int, int> class LBT, int EPI>
__device__ __forceinline__ void mfma_gemm_256p8_sk(const CoreParams& P, const SkParams& S) {
  constexpr int BM = 256, BN = 256, HR = 128;
  constexpr int SMEM = 8 * HR * BK;  // 128 KB, as mfma_gemm_256p8
  constexpr int FM = 8, FN = 4, NF = FM * FN;
  __shared__ __attribute__((aligned(16))) short smem[SMEM];

  const int tid = threadIdx.x;
  const int G = gridDim.x;
  const int lid = xcd_remap(blockIdx.x, G);
  const int tiles_m = (P.M + BM - 1) / BM, tiles_n = (P.N + BN - 1) / BN;
  int it = sk_start(lid, S.total, G);
  const int end = sk_start(lid + 1, S.total, G);
  f4v acc[FM][FN];
  while (it < end) {
    const int tile = it / S.ipt;
    const int k0 = it - tile * S.ipt;
    const int k1 = S.ipt < k0 + (end - it) ? S.ipt : k0 + (end - it);
    int tm, tn;
    tile256_coords(tile, tiles_m, tiles_n, tm, tn);
    const int m0 = tm * BM, n0 = tn * BN;
    const int kend = k1 * BK < P.K ? k1 * BK : P.K;
    P8Loop<LAT, LBT>::run(P, m0, n0, k0 * BK, kend, smem, acc);
    bool finish = true;  // this workgroup runs the tile's epilogue (one call site: register budget)
    if (k0 != 0) {
      // contributor: its range STARTS inside this tile, so this is its first segment and the
      // only partial it ever stores (slot lid); publish it, then the ticket (release)
      // the lane offset passes through an empty asm so its 32 store addresses are formed
      // here, not hoisted out of the segment loop (64 live VGPRs -> spills)
      uint32_t off = (uint32_t)(lid * NF * 512 + tid) * 16u;
      asm volatile("" : "+v"(off));
      char* dst = reinterpret_cast<char*>(S.part) + off;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) *reinterpret_cast<f4v*>(dst + (i * FN + j) * 512 * 16) = acc[i][j];
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(S.ticket + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      finish = false;
    } else if (k1 != S.ipt) {
      // owner of a split tile: wait for the other contributors, add their partials in order
      const int last = sk_owner_of(tile * S.ipt + S.ipt - 1, S.total, G);
      if (tid == 0) {
        // bounded: a contributor that never arrives (it cannot: the grid is <= the CU count,
        // every range non-empty, and no other stream-K launch runs beside this one) ends the
        // wait after ~0.2 s with an error word for the host instead of hanging the GPU
        const int want = last - lid;
        int spins = 0;
        while (__hip_atomic_load(S.ticket + tile, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
          __builtin_amdgcn_s_sleep(8);
          if (++spins == (1 << 20)) {
            __hip_atomic_store(S.ticket + S.err_index, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        __hip_atomic_store(S.ticket + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      for (int w = lid + 1; w <= last; ++w) {
        uint32_t off = (uint32_t)(w * NF * 512 + tid) * 16u;
        asm volatile("" : "+v"(off));
        const char* src = reinterpret_cast<const char*>(S.part) + off;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          f4v v[FN];
#pragma unroll
          for (int j = 0; j < FN; ++j) v[j] = *reinterpret_cast<const f4v*>(src + (i * FN + j) * 512 * 16);
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] += v[j];
          asm volatile("" ::: "memory");  // at most one fragment row of loads in flight
        }
      }
    }
    if (finish) gemm_epilogue<BM, BN, 2, 4, EPI, SMEM, 1, FM, FN, true>(P, acc, smem, m0, n0, tm, tid);
    __syncthreads();  // the next segment's DMA overwrites the epilogue's C staging
    it += k1 - k0;
  }
}

// 256 x 128 x 64 variant for GEMMs whose 256 x 256 grid does not fill whole rounds of the chip
// but whose 256 x 128 grid does (BERT-base at M = 8192: N = 3072 -> 768 tiles = 3 rounds, where
// 256 x 256 gives 384 = 1.5).  Same two staggered 4-wave groups; ONE phase per K tile (the
// whole 256 x 128 tile, 32 MFMAs per wave: waves 4 (M) x 2 (N), 64 x 64 each) and THREE LDS
// buffers of one K tile (A 32 KB + B 16 KB each, 144 KB): K tile t+2 is restaged into the
// buffer K tile t-1 used, one phase after its reads retired, and ONE counted vmcnt(6) per K
// tile (t+2's six loads per thread still in flight) completes t+1 before the phase that reads it.
template <template <int, int, int> class LAT, template <int, int, int> class LBT, int EPI>
__device__ __forceinline__ void mfma_gemm_256x128(const CoreParams& P) {
  constexpr int BM = 256, BN = 128, NT = 512, WM = 4, WN = 2;
  constexpr int AT = BM * BK, BT = BN * BK, ST = AT + BT;  // shorts per buffer
  constexpr int SMEM = 3 * ST;                              // 144 KB
  static_assert(SMEM >= BM * EpiLayout<BN>::LD, "C staging must fit the operand image");
  using LA = LAT<BM, 4, NT>;
  using LB = LBT<BN, 2, NT>;
  static_assert(!loader_stateful<LA>::value && !loader_stateful<LB>::value, "stateless loaders only");
  constexpr bool A_KC = LA::KC, B_KC = LB::KC;
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;  // 4 x 4
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
  const int nk = (kend - kbeg + BK - 1) / BK;

  const LA la(P, true, m0, tid);
  const LB lb(P, false, n0, tid);
  const auto ra = loader_rsrc(la);
  const auto rb = loader_rsrc(lb);
  auto dma = [&](int t) {
    const int k0 = kbeg + t * BK;
    short* As = smem + (t % 3) * ST;
    short* Bs = As + AT;
#pragma unroll
    for (int i = 0; i < 4; ++i) CA_DMA_CHUNK(LA, la, ra, i, k0, As + (i * NT + wave * 64) * 8);
#pragma unroll
    for (int i = 0; i < 2; ++i) CA_DMA_CHUNK(LB, lb, rb, i, k0, Bs + (i * NT + wave * 64) * 8);
  };

  f4v acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) dma(0);
  if (nk > 1) {
    dma(1);
    vm_wait<6>();
  } else {
    vm_wait<0>();
  }
  bar256();
  if (grp == 1) bar256();
  for (int t = 0; t < nk; ++t) {
    const short* As = smem + (t % 3) * ST;
    const short* Bs = As + AT;
    bf16x8 af[FM][2], bfr[FN][2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j][kk] = read_frag_sw<BN, B_KC>(Bs, wn * (BN / WN) + j * 16, kk * 32, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i][kk] = read_frag_sw<BM, A_KC>(As, wm * (BM / WM) + i * 16, kk * 32, lane);
    }
    lgkm_wait0();
    if (t + 2 < nk) {  // into the buffer K tile t-1 used (its reads retired before the last barrier)
      dma(t + 2);
      vm_wait<6>();
    } else {
      vm_wait<0>();
    }
    bar256();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j][kk], af[i][kk], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    bar256();
  }
  if (grp == 0) bar256();
  __syncthreads();
  gemm_epilogue<BM, BN, WM, WN, EPI, SMEM, 1>(P, acc, smem, m0, n0, tm, tid);
}

}  // namespace ca
