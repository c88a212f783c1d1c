// GEMM core whose A operand is PRODUCED in the load path by a BatchNorm transform
// (gfx950 / CDNA4): the ResNet-50 "BN folded into the consuming convolution" kernels.
//
//   C[M, N] = X(A-sources)[M, K] * B        X = per-element BN transform, per-K coefficients
//
// Why: in a bottleneck block every BatchNorm pass is a full read + write of an activation
// tensor, and the 1x1 convolution that consumes its output reads it straight back.  Folding
// the BN pass into the convolution's operand fetch removes that re-read (and a launch):
//
//   XA_BN_BWD       dz = A[k] * g + B[k] * z + D[k],  g = dy * relu'(mask)
//                   the BN(+ReLU) backward apply (bn.hip bn_bwd_apply_kernel) feeding the
//                   input-gradient GEMM of the 1x1 conv that produced z (conv3 / conv1 dgrad)
//   XA_BN_RELU      y = relu(z * scale[k] + shift[k])                  (forward, bn -> conv)
//   XA_BN_RES_RELU  y = relu(z * scale[k] + shift[k] + r)              (bn3 + identity residual)
//   XA_BN_RESBN_RELU y = relu(z * scale[k] + shift[k] + bf16(r * rscale[k] + rshift[k]))
//                   (bn3 + a projection shortcut whose own BN is applied on the fly, exactly
//                   as bn.hip bn_apply_resbn_kernel)
//
// The transformed tile is ALSO written to global memory (`side`, plus the forward's ReLU
// bitmask) by the blocks of the first N tile, so the tensors the rest of the step reads
// (the weight gradient's operand, the backward's ReLU mask) exist exactly as the unfused
// passes would have written them -- bit for bit: the arithmetic below is the BN kernels'.
//
// Pipeline (4 waves, 128 x BN tile, one LDS stage, several blocks per CU):
//   * A is register-staged: the next K step's 16-B source chunks (and coefficients, mask
//     bytes) are loaded into VGPRs while this step's MFMAs run, then transformed and written
//     to LDS with the swizzle read_frag_sw expects (phys chunk = logical ^ (row & 7));
//   * B (the weights, L2-resident) is register-staged the same way.  No LDS-DMA here: with
//     a DMA in flight the compiler's waitcnt pass cannot tell which LDS bytes it writes and
//     drains the A prefetch before the first LDS read of every step;
//   * all loads and side stores are buffer operations with a range check (rows past M or K
//     read zeros / are dropped), so no vector-memory operation sits behind a branch.
// Epilogues are the shared gemm_epilogue (BN statistics, residual-gated beta, ...).
#pragma once
#include "ca_gemm_prw.h"

namespace ca {

enum XaMode { XA_BN_RELU = 0, XA_BN_RES_RELU = 1, XA_BN_BWD = 2, XA_BN_RESBN_RELU = 3 };

struct XaParams {
  const bf16_t* src0;      // z (forward) / dy (backward)                [M][K], row stride lda
  const bf16_t* src1;      // residual r (XA_BN_RES_RELU) / z (XA_BN_BWD) [M][K], row stride lda
  const uint8_t* mask_in;  // XA_BN_BWD: ReLU bitmask [M][K/8] or null (no ReLU)
  const float* c0;         // scale (forward) / A (backward)  [K]
  const float* c1;         // shift (forward) / B (backward)  [K]
  const float* c2;         // D (backward) / rscale (XA_BN_RESBN_RELU) [K]
  const float* c3;         // rshift (XA_BN_RESBN_RELU)                [K]
  bf16_t* side;            // transformed A [M][K] (row stride lda), written by N tile 0; may be null
  uint8_t* mask_out;       // forward: ReLU bitmask of the transformed A [M][K/8]; may be null
};

template <int XM>
struct XaTraits {
  static constexpr bool TWO = XM != XA_BN_RELU;        // second source tensor
  static constexpr bool MASK_IN = XM == XA_BN_BWD;      // backward ReLU gate
  static constexpr int NCOEF = XM == XA_BN_BWD ? 3 : (XM == XA_BN_RESBN_RELU ? 4 : 2);
};

// NT = 256 (4 waves, 2 x 2) or 512 (8 waves, 2 x 4: half the registers per lane, so two
// workgroups -- 16 waves -- per CU keep twice the loads in flight)
template <int BM, int BN, bool B_KC, int EPI, int XM, int NT = 256>
__device__ __forceinline__ void mfma_gemm_xa(const CoreParams& P, const XaParams& X) {
  constexpr int WM = 2, WN = NT / 128;
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;
  static_assert(FN >= 1, "at least one 16-column fragment per wave");
  constexpr int A_ELEMS = BM * BK, B_ELEMS = BN * BK;
  constexpr int STAGE = A_ELEMS + B_ELEMS;
  constexpr int EPI_LD = EpiLayout<BN>::LD;
  constexpr int SRED = 2 * (NT / (BN / 8)) * BN * 2;  // two fp32 statistics rows per thread group
  constexpr int SMEM0 = (STAGE > BM * EPI_LD ? STAGE : BM * EPI_LD);
  constexpr int SMEM = SMEM0 > SRED ? SMEM0 : SRED;
  constexpr int CPA = A_ELEMS / 8 / NT;  // A chunks (16 B) per thread and K step
  constexpr int CPB = B_ELEMS / 8 / NT;
  constexpr int RSTEP = NT / 8;          // tile rows between a thread's A chunks
  using T = XaTraits<XM>;
  static_assert(A_ELEMS % (8 * NT) == 0 && B_ELEMS % (8 * NT) == 0, "tile chunks must divide threads");
  __shared__ __attribute__((aligned(16))) short smem[SMEM];
  short* const As = smem;
  short* const Bs = smem + A_ELEMS;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_n = (P.N + BN - 1) / BN;
  const BlkPos bp = blk_pos(P);
  const int tm = bp.tile / tiles_n, tn = bp.tile % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = (P.K + BK - 1) / BK;
  const int K8 = P.K >> 3;

  // B: the whole weight matrix is one buffer resource (KC: [N][K] rows, NC: [K][N] rows);
  // rows past its end read zeros.  A chunk's k / column beyond K / N only feeds products with
  // a zero A element or output columns that are never stored.
  const auto rbw = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(P.B), (short)0,
                                                     (int)buf_span((long)(B_KC ? P.N : P.K) * P.ldb * 2), 0x00020000);
  s8v bw[CPB];
  auto b_coord = [&](int i, int& lrow, int& lcol) {  // chunk i of this thread in the B tile
    const int c = tid + i * NT;
    if constexpr (B_KC) {
      lrow = c >> 3;                   // n
      lcol = c & 7;                    // 8-k group
    } else {
      lrow = c / (BN / 8);             // k
      lcol = c % (BN / 8);             // 8-n group
    }
  };

  // A geometry: thread tid owns logical 8-channel group c8 = tid & 7 of rows (tid >> 3) + RSTEP i
  const int arow = tid >> 3, c8 = tid & 7;
  const long rows_left = (long)P.M - m0;
  const uint32_t span = buf_span(rows_left * P.lda * 2);
  const auto r0s = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(X.src0 + (long)m0 * P.lda), (short)0,
                                                     (int)span, 0x00020000);
  const auto r1s = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>((T::TWO ? X.src1 : X.src0) + (long)m0 * P.lda), (short)0, (int)span, 0x00020000);
  const uint32_t mspan = buf_span(rows_left * K8);
  const auto rms = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(X.mask_in ? X.mask_in + (long)m0 * K8 : reinterpret_cast<const uint8_t*>(ca_zero16)),
      (short)0, X.mask_in ? (int)mspan : 0, 0x00020000);
  // side outputs: buffer stores through resources that are empty (num_records 0: every store
  // dropped) unless this block writes them -- every thread issues the same vector-memory
  // stream whatever its tile, so the compiler's and our counted waits stay exact (a store
  // behind a branch makes the waitcnt pass drain to vmcnt(0) before the LDS reads)
  const bool write_side = tn == 0;
  const auto rside = __builtin_amdgcn_make_buffer_rsrc(
      write_side && X.side ? X.side + (long)m0 * P.lda : const_cast<bf16_t*>(ca_zero16), (short)0,
      write_side && X.side ? (int)span : 0, 0x00020000);
  const auto rmout = __builtin_amdgcn_make_buffer_rsrc(
      write_side && X.mask_out ? X.mask_out + (long)m0 * K8 : reinterpret_cast<uint8_t*>(ca_zero16), (short)0,
      write_side && X.mask_out ? (int)mspan : 0, 0x00020000);

  s8v a0[CPA], a1[CPA];
  uint32_t mb[CPA];
  f4v cf[T::NCOEF][2];

  auto gload = [&](int t) {
    const int k = t * BK + 8 * c8;
    const int kc = k < P.K ? k : P.K - 8;  // K tail: a valid address, zeroed after the transform
#pragma unroll
    for (int i = 0; i < CPA; ++i) {
      const uint32_t off = (uint32_t)(((long)(arow + i * RSTEP) * P.lda + kc) * 2);
      a0[i] = __builtin_bit_cast(s8v, __builtin_amdgcn_raw_buffer_load_b128(r0s, (int)off, 0, 0));
      if constexpr (T::TWO) a1[i] = __builtin_bit_cast(s8v, __builtin_amdgcn_raw_buffer_load_b128(r1s, (int)off, 0, 0));
      if constexpr (T::MASK_IN)
        mb[i] = __builtin_amdgcn_raw_buffer_load_b8(rms, (int)((arow + i * RSTEP) * K8 + (kc >> 3)), 0, 0);
    }
#pragma unroll
    for (int i = 0; i < CPB; ++i) {
      int lr, lc;
      b_coord(i, lr, lc);
      const long off = B_KC ? (long)(n0 + lr) * P.ldb + t * BK + 8 * lc
                            : (long)(t * BK + lr) * P.ldb + (n0 + 8 * lc < P.N ? n0 + 8 * lc : P.N - 8);
      bw[i] = __builtin_bit_cast(s8v, __builtin_amdgcn_raw_buffer_load_b128(rbw, (int)(off * 2), 0, 0));
    }
    const float* cs[4] = {X.c0, X.c1, X.c2, X.c3};
#pragma unroll
    for (int q = 0; q < T::NCOEF; ++q) {
      cf[q][0] = *reinterpret_cast<const f4v*>(cs[q] + kc);
      cf[q][1] = *reinterpret_cast<const f4v*>(cs[q] + kc + 4);
    }
  };

  auto transform_store = [&](int t) {
    const int k = t * BK + 8 * c8;
    const bool kok = k < P.K;
#pragma unroll
    for (int i = 0; i < CPA; ++i) {
      const int row = arow + i * RSTEP;
      s8v o;
      uint32_t bits = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float c0 = cf[0][j >> 2][j & 3], c1 = cf[1][j >> 2][j & 3];
        float v;
        if constexpr (XM == XA_BN_BWD) {
          // bn_bwd_apply_kernel: d gated by the ReLU bit, then A*d + B*x + D
          float d = bf2f((bf16_t)a0[i][j]);
          if (X.mask_in) d = ((mb[i] >> j) & 1u) ? d : 0.f;
          const float c2 = cf[2][j >> 2][j & 3];
          v = bn_bwd_affine(c0, d, c1, bf2f((bf16_t)a1[i][j]), c2);
        } else {
          // bn_apply_kernel<true, RES>: z*scale + shift (+ r), ReLU, bit = y > 0
          float z = bn_affine(bf2f((bf16_t)a0[i][j]), c0, c1);
          if constexpr (XM == XA_BN_RES_RELU) z += bf2f((bf16_t)a1[i][j]);
          if constexpr (XM == XA_BN_RESBN_RELU) {
            // the shortcut BN output rounded to bf16 as if stored (bn_apply_resbn_kernel)
            const float idn = bf2f(f2bf(bn_affine(bf2f((bf16_t)a1[i][j]), cf[2][j >> 2][j & 3], cf[3][j >> 2][j & 3])));
            z = bn_affine(bf2f((bf16_t)a0[i][j]), c0, c1) + idn;
          }
          z = fmaxf(z, 0.f);
          bits |= (z > 0.f ? 1u : 0u) << j;
          v = z;
        }
        o[j] = kok ? (short)f2bf(v) : (short)0;
      }
      *reinterpret_cast<s8v*>(As + row * BK + ((c8 ^ (row & 7)) << 3)) = o;
      // rows past M and the K tail land beyond the resource's range: dropped by the hardware
      const uint32_t soff = kok ? (uint32_t)(((long)row * P.lda + k) * 2) : span;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rside, (int)soff, 0, 0);
      if constexpr (XM != XA_BN_BWD)
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)bits, rmout, kok ? (int)(row * K8 + (k >> 3)) : (int)mspan, 0,
                                             0);
    }
#pragma unroll
    for (int i = 0; i < CPB; ++i) {  // B chunks at the swizzled slots read_frag_sw reads
      int lr, lc;
      b_coord(i, lr, lc);
      short* dst = B_KC ? Bs + lr * BK + ((lc ^ (lr & 7)) << 3) : Bs + lr * BN + ((lc ^ nc_swz<BN>(lr)) << 3);
      *reinterpret_cast<s8v*>(dst) = bw[i];
    }
  };

  f4v acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) gload(0);
  for (int t = 0; t < nk; ++t) {
    transform_store(t);            // the stage is free: every wave passed the closing barrier of t - 1
    if (t + 1 < nk) gload(t + 1);  // next step's operands in flight during this step's MFMAs
    lgkm_wait0();
    bar256();
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = read_frag_sw<BM, true>(As, wm * (BM / WM) + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = read_frag_sw<BN, B_KC>(Bs, wn * (BN / WN) + j * 16, kk, lane);
      mfma_acc<FM, FN>(acc, af, bfr);
    }
    lgkm_wait0();
    bar256();
  }
  vm_wait<0>();
  gemm_epilogue<BM, BN, WM, WN, EPI, SMEM, 1>(P, acc, smem, m0, n0, tm, tid);
}

// ----------------------------------------------------------------------------------------
// The same GEMM on 128 x BN tiles with 16 waves and the raw operands of TWO K tiles in flight.
// One 16-wave workgroup per CU with the one-deep pipeline above keeps only one 32-KB raw K tile
// per CU on the way from HBM -- the latency-bandwidth product caps that at ~4 TB/s (measured:
// the stage-3 folded dgrad 3.03 ms vs 2.84 for the passes it replaces, docs/performance.md).
// Here the BN coefficients of the whole K range are staged in LDS once (K <= XA_DEEP_KMAX),
// which frees the registers of a second A / B / mask staging set: tile t + 2's loads are issued
// right after tile t's transform, so tiles t + 1 and t + 2 are in flight during tile t's MFMAs.
// The loop is unrolled by two so every staging set is a compile-time register set.
// Arithmetic (transform, K order, epilogue) is mfma_gemm_xa's: the outputs are bit-identical.
constexpr int XA_DEEP_KMAX = 2048;

template <int BN, bool B_KC, int EPI, int XM>
__device__ __forceinline__ void mfma_gemm_xa_deep(const CoreParams& P, const XaParams& X) {
  constexpr int BM = 128, NT = 1024, WM = 2, WN = NT / 128;
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;
  static_assert(FN >= 1, "at least one 16-column fragment per wave");
  constexpr int A_ELEMS = BM * BK, B_ELEMS = BN * BK;
  constexpr int STAGE = A_ELEMS + B_ELEMS;
  constexpr int EPI_LD = EpiLayout<BN>::LD;
  constexpr int SRED = 2 * (NT / (BN / 8)) * BN * 2;
  constexpr int SMEM0 = (STAGE > BM * EPI_LD ? STAGE : BM * EPI_LD);
  constexpr int SMEM = SMEM0 > SRED ? SMEM0 : SRED;
  constexpr int CPB = B_ELEMS / 8 / NT;
  using T = XaTraits<XM>;
  static_assert(A_ELEMS == 8 * NT, "one A chunk per thread and K step");
  static_assert(B_ELEMS % (8 * NT) == 0, "B chunks must divide the threads");
  __shared__ __attribute__((aligned(16))) short smem[SMEM];
  __shared__ __attribute__((aligned(16))) float coefs[T::NCOEF * XA_DEEP_KMAX];
  short* const As = smem;
  short* const Bs = smem + A_ELEMS;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_n = (P.N + BN - 1) / BN;
  const BlkPos bp = blk_pos(P);
  const int tm = bp.tile / tiles_n, tn = bp.tile % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = (P.K + BK - 1) / BK;
  const int K8 = P.K >> 3;

  {  // the coefficients of every k, once (the host guarantees K <= XA_DEEP_KMAX)
    const float* cs[4] = {X.c0, X.c1, X.c2, X.c3};
#pragma unroll
    for (int q = 0; q < T::NCOEF; ++q)
      for (int k = tid; k < P.K; k += NT) coefs[q * XA_DEEP_KMAX + k] = cs[q][k];
  }

  const auto rbw = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(P.B), (short)0,
                                                     (int)buf_span((long)(B_KC ? P.N : P.K) * P.ldb * 2), 0x00020000);
  auto b_coord = [&](int i, int& lrow, int& lcol) {
    const int c = tid + i * NT;
    if constexpr (B_KC) {
      lrow = c >> 3;
      lcol = c & 7;
    } else {
      lrow = c / (BN / 8);
      lcol = c % (BN / 8);
    }
  };
  const int arow = tid >> 3, c8 = tid & 7;
  const long rows_left = (long)P.M - m0;
  const uint32_t span = buf_span(rows_left * P.lda * 2);
  const auto r0s = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(X.src0 + (long)m0 * P.lda), (short)0,
                                                     (int)span, 0x00020000);
  const auto r1s = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>((T::TWO ? X.src1 : X.src0) + (long)m0 * P.lda), (short)0, (int)span, 0x00020000);
  const uint32_t mspan = buf_span(rows_left * K8);
  const auto rms = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(X.mask_in ? X.mask_in + (long)m0 * K8 : reinterpret_cast<const uint8_t*>(ca_zero16)),
      (short)0, X.mask_in ? (int)mspan : 0, 0x00020000);
  const bool write_side = tn == 0;
  const auto rside = __builtin_amdgcn_make_buffer_rsrc(
      write_side && X.side ? X.side + (long)m0 * P.lda : const_cast<bf16_t*>(ca_zero16), (short)0,
      write_side && X.side ? (int)span : 0, 0x00020000);
  const auto rmout = __builtin_amdgcn_make_buffer_rsrc(
      write_side && X.mask_out ? X.mask_out + (long)m0 * K8 : reinterpret_cast<uint8_t*>(ca_zero16), (short)0,
      write_side && X.mask_out ? (int)mspan : 0, 0x00020000);

  // two staging sets, indexed by literal 0 / 1 only (the loop below is unrolled by two)
  s8v a0[2], a1[2], bw[2][CPB];
  uint32_t mb[2];

  auto gload = [&](int t, const int S) {
    const int k = t * BK + 8 * c8;
    const int kc = k < P.K ? k : P.K - 8;
    const uint32_t off = (uint32_t)(((long)arow * P.lda + kc) * 2);
    a0[S] = __builtin_bit_cast(s8v, __builtin_amdgcn_raw_buffer_load_b128(r0s, (int)off, 0, 0));
    if constexpr (T::TWO) a1[S] = __builtin_bit_cast(s8v, __builtin_amdgcn_raw_buffer_load_b128(r1s, (int)off, 0, 0));
    if constexpr (T::MASK_IN) mb[S] = __builtin_amdgcn_raw_buffer_load_b8(rms, (int)(arow * K8 + (kc >> 3)), 0, 0);
#pragma unroll
    for (int i = 0; i < CPB; ++i) {
      int lr, lc;
      b_coord(i, lr, lc);
      const long boff = B_KC ? (long)(n0 + lr) * P.ldb + t * BK + 8 * lc
                             : (long)(t * BK + lr) * P.ldb + (n0 + 8 * lc < P.N ? n0 + 8 * lc : P.N - 8);
      bw[S][i] = __builtin_bit_cast(s8v, __builtin_amdgcn_raw_buffer_load_b128(rbw, (int)(boff * 2), 0, 0));
    }
  };

  auto transform_store = [&](int t, const int S) {
    const int k = t * BK + 8 * c8;
    const bool kok = k < P.K;
    const int kc = kok ? k : P.K - 8;
    f4v cf[T::NCOEF][2];
#pragma unroll
    for (int q = 0; q < T::NCOEF; ++q) {
      cf[q][0] = *reinterpret_cast<const f4v*>(coefs + q * XA_DEEP_KMAX + kc);
      cf[q][1] = *reinterpret_cast<const f4v*>(coefs + q * XA_DEEP_KMAX + kc + 4);
    }
    s8v o;
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float c0 = cf[0][j >> 2][j & 3], c1 = cf[1][j >> 2][j & 3];
      float v;
      if constexpr (XM == XA_BN_BWD) {
        float d = bf2f((bf16_t)a0[S][j]);
        if (X.mask_in) d = ((mb[S] >> j) & 1u) ? d : 0.f;
        v = bn_bwd_affine(c0, d, c1, bf2f((bf16_t)a1[S][j]), cf[2][j >> 2][j & 3]);
      } else {
        float z = bn_affine(bf2f((bf16_t)a0[S][j]), c0, c1);
        if constexpr (XM == XA_BN_RES_RELU) z += bf2f((bf16_t)a1[S][j]);
        if constexpr (XM == XA_BN_RESBN_RELU) {
          const float idn = bf2f(f2bf(bn_affine(bf2f((bf16_t)a1[S][j]), cf[2][j >> 2][j & 3], cf[3][j >> 2][j & 3])));
          z = bn_affine(bf2f((bf16_t)a0[S][j]), c0, c1) + idn;
        }
        z = fmaxf(z, 0.f);
        bits |= (z > 0.f ? 1u : 0u) << j;
        v = z;
      }
      o[j] = kok ? (short)f2bf(v) : (short)0;
    }
    *reinterpret_cast<s8v*>(As + arow * BK + ((c8 ^ (arow & 7)) << 3)) = o;
    const uint32_t soff = kok ? (uint32_t)(((long)arow * P.lda + k) * 2) : span;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rside, (int)soff, 0, 0);
    if constexpr (XM != XA_BN_BWD)
      __builtin_amdgcn_raw_buffer_store_b8((uint8_t)bits, rmout, kok ? (int)(arow * K8 + (k >> 3)) : (int)mspan, 0, 0);
#pragma unroll
    for (int i = 0; i < CPB; ++i) {
      int lr, lc;
      b_coord(i, lr, lc);
      short* dst = B_KC ? Bs + lr * BK + ((lc ^ (lr & 7)) << 3) : Bs + lr * BN + ((lc ^ nc_swz<BN>(lr)) << 3);
      *reinterpret_cast<s8v*>(dst) = bw[S][i];
    }
  };

  f4v acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  // Every load is issued unconditionally (past the last tile: the last tile again, never used)
  // and the loop body has no branch, so the compiler's waitcnt pass sees one static stream of
  // vector-memory operations and waits for exactly the set it is about to read -- a branch
  // around a refill merges two counter states and it falls back to vmcnt(0) (checked in the .s).
  auto step = [&](int t, const int S) {
    transform_store(t, S);                    // the stage is free: every wave passed t - 1's closing barrier
    gload(t + 2 < nk ? t + 2 : nk - 1, S);    // refill this set: tiles t + 1 and t + 2 in flight now
    lgkm_wait0();
    bar256();
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = read_frag_sw<BM, true>(As, wm * (BM / WM) + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = read_frag_sw<BN, B_KC>(Bs, wn * (BN / WN) + j * 16, kk, lane);
      mfma_acc<FM, FN>(acc, af, bfr);
    }
    lgkm_wait0();
    bar256();
  };

  gload(0, 0);  // (the host guarantees K >= 8: nk >= 1)
  gload(nk > 1 ? 1 : 0, 1);
  __syncthreads();  // coefficients staged
  int t = 0;
#pragma unroll 1
  for (; t + 1 < nk; t += 2) {
    step(t, 0);
    step(t + 1, 1);
  }
  if (t < nk) step(t, 0);
  vm_wait<0>();
  gemm_epilogue<BM, BN, WM, WN, EPI, SMEM, 1>(P, acc, smem, m0, n0, tm, tid);
}

// ----------------------------------------------------------------------------------------
// XA_BN_BWD with the WEIGHT gradient in the same pass (ResNet stage-1 1x1 convolutions:
// conv3, K = 4c = 256 -> N = c = 64; conv1, K = c = 64 -> N = 4c = 256).  The unfused
// schedule writes dz (the BN-backward apply, [M][K]) and reads it back in the split-K
// weight-gradient GEMM (and, at the short-K conv1, in a separate input-gradient GEMM);
// here each workgroup owns a contiguous range of 128-row tiles and, while a transformed dz
// chunk is in LDS, runs BOTH products on it:
//
//   dx[m, n]  = sum_k dz[m, k] W[k, n]        (per tile; the dgrad epilogues: BN statistics,
//                                             residual-gated / plain beta accumulate)
//   dW[k, n] += sum_m dz[m, k] y[m, n]        (accumulated in registers over ALL the
//                                             workgroup's tiles; y = the conv's input)
//
// so dz never reaches memory.  Steps: KS K chunks x NC N chunks of 64 (KS == 1 or NC == 1,
// KS * NC <= 4: the dW block K x N <= 16K floats = 64 per thread).  With NC > 1 the dz tile
// (K = 64) is transformed once and reused by every N chunk; each N chunk runs its epilogue.
// dW leaves as one fp32 slab per workgroup ([K][N], deterministic; ca_splitk_reduce sums
// them).  The dz chunk is read twice from one LDS image: as the dgrad A operand (row m, 8
// consecutive k) and, through ds_read_b64_tr_b16, as the wgrad A operand (row k, 8
// consecutive m) -- the read_frag_sw N-contiguous read with this image's (m & 7) swizzle.
//
// BN = 64 with 4 waves (stage 1), or BN = 128 with 8 waves (stage 2 conv3: K = 512 -> N = 128,
// a 512 x 128 dW block = 128 fp32 per lane, one workgroup per CU): waves 2 (M) x BN/32 (N) for
// the dgrad tile, 2 (k) x BN/32 (n) 32 x 32 blocks of each dW chunk.
template <int EPI, int KS, int NC, int BN = 64, int NT = 256, int BM = 128>
__device__ __forceinline__ void mfma_gemm_xa_dw(const CoreParams& P, const XaParams& X, const bf16_t* Y, long ldy,
                                                float* ws, int tiles_per_block) {
  static_assert((KS == 1 || NC == 1) && KS >= 1 && NC >= 1, "K chunks or N chunks, not both");
  static_assert((BN == 64 && (NT == 256 || NT == 512)) || (BN == 128 && NT == 512), "64 columns (4 or 8 waves), 128 (8)");
  static_assert(BM == 128 || BM == 64, "128- or 64-row tiles");
  constexpr int WM = 2, WN = NT / 64 / WM;
  constexpr int WNB = BN / WN, FNW = WNB / 16;  // a wave's dW / dgrad columns, its 16-wide fragments
  static_assert(KS * NC * 8 * FNW <= 64 * (NT / 256), "dW block per lane: <= 64 fp32 (4 waves) / 128 (8 waves)");
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;  // dgrad: 4 x 2 fragments per wave
  constexpr int A_ELEMS = BM * BK, B_ELEMS = BK * BN, Y_ELEMS = BM * BN;
  constexpr int CPA = A_ELEMS / 8 / NT, CPB = B_ELEMS / 8 / NT, CPY = Y_ELEMS / 8 / NT;
  constexpr int RSTEP = NT / 8;
  constexpr int K = KS * BK, N = NC * BN, STEPS = KS * NC;
  // LDS: As (dz chunk) | Bs (W chunk) | Ys (y chunk) | coefficients.  The epilogue stages
  // C and its statistics rows in Bs + Ys (free between the steps' barriers), never in As.
  // (the statistics epilogues reduce up to three fp32 rows per thread group: 3 * NT/(BN/8) * BN floats)
  constexpr int SRED = 3 * (NT / (BN / 8)) * BN * 2;
  constexpr int EPI_SH = (B_ELEMS + Y_ELEMS) > SRED ? (B_ELEMS + Y_ELEMS) : SRED;
  static_assert(BM * EpiLayout<BN>::LD <= EPI_SH, "C staging must fit Bs + Ys");
  __shared__ __attribute__((aligned(16))) short smem[A_ELEMS + EPI_SH + 3 * K * 2];
  short* const As = smem;
  short* const Bs = smem + A_ELEMS;
  short* const Ys = Bs + B_ELEMS;
  float* const Cf = reinterpret_cast<float*>(Bs + EPI_SH);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_m = (P.M + BM - 1) / BM;
  const int t_beg = blockIdx.x * tiles_per_block;
  int t_end = t_beg + tiles_per_block;
  if (t_end > tiles_m) t_end = tiles_m;
  constexpr int K8 = K >> 3;

  const auto rbw = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(P.B), (short)0,
                                                     (int)buf_span((long)K * P.ldb * 2), 0x00020000);
  const int arow = tid >> 3, c8 = tid & 7;

  f4v accw[STEPS][2][FNW];  // dW: per (K chunk, N chunk) step, a 32 (k) x WNB (n) block per wave
#pragma unroll
  for (int c = 0; c < STEPS; ++c)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < FNW; ++j) accw[c][i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  for (int i = tid; i < 3 * K; i += NT) {
    const int q = i / K, k = i - q * K;
    Cf[i] = (q == 0 ? X.c0 : (q == 1 ? X.c1 : X.c2))[k];
  }

  s8v a0[CPA], a1[CPA], bw[CPB], yv[CPY];
  uint32_t mb[CPA];

  // per-tile operand windows (buffer resources; rows past M read zeros), switched to the NEXT
  // tile during the last step of the current one so that tile's first loads fly during this
  // tile's last MFMAs and its epilogue
  __amdgpu_buffer_rsrc_t r0s, r1s, rms, rys;
  auto set_tile = [&](int t) {
    const int mt = t * BM;
    const long rl = (long)P.M - mt;
    const uint32_t span = buf_span(rl * P.lda * 2);
    r0s = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(X.src0 + (long)mt * P.lda), (short)0, (int)span,
                                            0x00020000);
    r1s = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(X.src1 + (long)mt * P.lda), (short)0, (int)span,
                                            0x00020000);
    rms = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(X.mask_in ? X.mask_in + (long)mt * K8 : reinterpret_cast<const uint8_t*>(ca_zero16)),
        (short)0, X.mask_in ? (int)buf_span(rl * K8) : 0, 0x00020000);
    rys = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(Y + (long)mt * ldy), (short)0,
                                            (int)buf_span(rl * ldy * 2), 0x00020000);
  };
  bool prefetched = false;

#pragma unroll 1
  for (int tm = t_beg; tm < t_end; ++tm) {
    const int m0 = tm * BM;
    if (!prefetched) set_tile(tm);

    auto load_a = [&](int t) {  // dz sources of K chunk t
      const int k = t * BK + 8 * c8;
#pragma unroll
      for (int i = 0; i < CPA; ++i) {
        const uint32_t off = (uint32_t)(((long)(arow + i * RSTEP) * P.lda + k) * 2);
        a0[i] = __builtin_bit_cast(s8v, __builtin_amdgcn_raw_buffer_load_b128(r0s, (int)off, 0, 0));
        a1[i] = __builtin_bit_cast(s8v, __builtin_amdgcn_raw_buffer_load_b128(r1s, (int)off, 0, 0));
        mb[i] = __builtin_amdgcn_raw_buffer_load_b8(rms, (int)((arow + i * RSTEP) * K8 + (k >> 3)), 0, 0);
      }
    };
    auto load_w = [&](int t, int nc) {  // W [K][N] rows k of chunk t, columns of chunk nc
#pragma unroll
      for (int i = 0; i < CPB; ++i) {
        const int c = tid + i * NT, lr = c / (BN / 8), lc = c % (BN / 8);
        const long off = (long)(t * BK + lr) * P.ldb + nc * BN + 8 * lc;
        bw[i] = __builtin_bit_cast(s8v, __builtin_amdgcn_raw_buffer_load_b128(rbw, (int)(off * 2), 0, 0));
      }
    };
    auto load_y = [&](int nc) {  // conv input rows of this tile, columns of chunk nc (rows past M: zeros)
#pragma unroll
      for (int i = 0; i < CPY; ++i) {
        const int c = tid + i * NT, lr = c / (BN / 8), lc = c % (BN / 8);
        yv[i] = __builtin_bit_cast(s8v, __builtin_amdgcn_raw_buffer_load_b128(
                                            rys, (int)(((long)lr * ldy + nc * BN + 8 * lc) * 2), 0, 0));
      }
    };
    auto store_a = [&](int t) {  // transform: dz = A*(dy*relu') + B*z + D  (bn_bwd_apply_kernel)
      const int k = t * BK + 8 * c8;
      f4v cf[3][2];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        cf[q][0] = *reinterpret_cast<const f4v*>(Cf + q * K + k);
        cf[q][1] = *reinterpret_cast<const f4v*>(Cf + q * K + k + 4);
      }
#pragma unroll
      for (int i = 0; i < CPA; ++i) {
        const int row = arow + i * RSTEP;
        s8v o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float d = bf2f((bf16_t)a0[i][j]);
          if (X.mask_in) d = ((mb[i] >> j) & 1u) ? d : 0.f;
          o[j] = (short)f2bf(
              bn_bwd_affine(cf[0][j >> 2][j & 3], d, cf[1][j >> 2][j & 3], bf2f((bf16_t)a1[i][j]), cf[2][j >> 2][j & 3]));
        }
        *reinterpret_cast<s8v*>(As + row * BK + ((c8 ^ (row & 7)) << 3)) = o;
      }
    };
    auto store_w = [&]() {
#pragma unroll
      for (int i = 0; i < CPB; ++i) {
        const int c = tid + i * NT, lr = c / (BN / 8), lc = c % (BN / 8);
        *reinterpret_cast<s8v*>(Bs + lr * BN + ((lc ^ nc_swz<BN>(lr)) << 3)) = bw[i];
      }
    };
    auto store_y = [&]() {
#pragma unroll
      for (int i = 0; i < CPY; ++i) {
        const int c = tid + i * NT, lr = c / (BN / 8), lc = c % (BN / 8);
        *reinterpret_cast<s8v*>(Ys + lr * BN + ((lc ^ nc_swz<BN>(lr)) << 3)) = yv[i];
      }
    };

    if (!prefetched) {
      load_y(0);
      load_a(0);
      load_w(0, 0);
    }
    prefetched = false;
    if (tm == t_beg) __syncthreads();  // the coefficient table is in LDS

    f4v acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
      const int t = s % KS, nc = s / KS;
      // stage this step's operands (the previous step's readers passed its closing barrier)
      if (NC == 1 || s == 0) store_a(t);
      store_w();
      if (t == 0) store_y();
      if (s + 1 < STEPS) {  // next step's loads fly during this step's MFMAs (and epilogue)
        const int t1 = (s + 1) % KS, n1 = (s + 1) / KS;
        if (NC == 1) load_a(t1);
        load_w(t1, n1);
        if (t1 == 0) load_y(n1);
      } else if (tm + 1 < t_end) {  // the next tile's first step
        set_tile(tm + 1);
        load_y(0);
        load_a(0);
        load_w(0, 0);
        prefetched = true;
      }
      lgkm_wait0();
      bar256();
      // dgrad: dx chunk += dz chunk (rows m) x W chunk (loops kept rolled: hoisting every
      // fragment read of the step would not fit next to the two accumulator sets)
#pragma unroll 1
      for (int kk = 0; kk < BK; kk += 32) {
        bf16x8 af[FM], bfr[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) af[i] = read_frag_sw<BM, true>(As, wm * (BM / WM) + i * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < FN; ++j) bfr[j] = read_frag_sw<BN, false>(Bs, wn * (BN / WN) + j * 16, kk, lane);
        mfma_acc<FM, FN>(acc, af, bfr);
      }
      // wgrad: dW (chunk t, chunk nc) += dz chunk^T (rows k) x y chunk (rows m), over the tile's rows
#pragma unroll 1
      for (int mk = 0; mk < BM; mk += 32) {
        bf16x8 dzt[2], yf[FNW];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          // N-contiguous read of the [m][k] dz image (chunk swizzle m & 7): row k, 8 consecutive m
          const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
          const int mr = mk + 8 * g + q;
          const int lc = ((wm * 32 + i * 16) >> 3) + (pp >> 1);
          const int sub = 4 * (pp & 1);
          const short* b0 = As + mr * BK + ((lc ^ (mr & 7)) << 3) + sub;
          const short* b1 = As + (mr + 4) * BK + ((lc ^ ((mr + 4) & 7)) << 3) + sub;
          s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(b0));
          s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(b1));
          dzt[i] = __builtin_bit_cast(bf16x8, s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
        }
#pragma unroll
        for (int j = 0; j < FNW; ++j) yf[j] = read_frag_sw<BN, false>(Ys, wn * WNB + j * 16, mk, lane);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < FNW; ++j)
            accw[s][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(yf[j], dzt[i], accw[s][i][j], 0, 0, 0);
      }
      lgkm_wait0();
      bar256();
      if (t == KS - 1) {  // dx chunk nc complete
        gemm_epilogue<BM, BN, WM, WN, EPI, EPI_SH, 1>(P, acc, Bs, m0, nc * BN, tm, tid);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
  // dW slab of this workgroup: accw[s][i][j][r] = dW[64 t + 32 wm + 16 i + (lane & 15)][64 nc + WNB wn + 16 j + 4 (lane >> 4) + r]
  float* slab = ws + (long)blockIdx.x * K * N;
#pragma unroll
  for (int s = 0; s < STEPS; ++s) {
    const int t = s % KS, nc = s / KS;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < FNW; ++j) {
        const int k = t * BK + wm * 32 + i * 16 + (lane & 15);
        const int n = nc * BN + wn * WNB + j * 16 + 4 * (lane >> 4);
        *reinterpret_cast<f4v*>(slab + (long)k * N + n) = accw[s][i][j];
      }
  }
}

// ----------------------------------------------------------------------------------------
// mfma_gemm_xa_dw with a deeper operand stream, for the shape that carries ResNet-50's
// stage-1 traffic (K = 4 x 64 -> N = 64, NC == 1: conv3 and the projection shortcut).  The
// form above keeps one K step of dz sources in flight per workgroup (~33 KB; two workgroups
// per CU) and runs at ~3.5 TB/s.  Here:
//   * the whole K x 64 weight block is copied to LDS once per workgroup (it is the same for
//     every tile), so the step stream carries only dy, z and the ReLU mask;
//   * the sources of step g + PD load while step g runs (PD register sets; set = step % PD,
//     static since KS % PD == 0), across tile boundaries: the next tile's y and first steps
//     are in flight during this tile's last steps and its epilogue;
//   * one buffer window per tensor covers the workgroup's tile range, so the "next tile"
//     past the range reads nothing (hardware range check) and no load sits behind a branch;
//   * the BN-statistics epilogue's operands (z, ReLU mask of the consuming BN) are loaded in
//     the stream BEFORE the next tile's sources: vmcnt retires in issue order, so a load
//     issued after them would make the epilogue wait for the next tile.
// The epilogue (bf16 dx, optional BN-backward statistics) is gemm_epilogue's arithmetic in
// its order, staged in As + Ys.  beta = 0, no residual / second BN: the host checks.
// Registers: PD = 1 fits two workgroups per CU (256); PD = 2 / 4 run one workgroup per CU
// (waves_per_eu(1)), with 2 / 4 steps (66 / 132 KB) in flight.
template <int EPI, int KS, int PD>
__device__ __forceinline__ void mfma_gemm_xa_dw_deep(const CoreParams& P, const XaParams& X, const bf16_t* Y,
                                                     long ldy, float* ws, int tiles_per_block) {
  static_assert(EPI == EPI_BF16 || EPI == EPI_BF16_BN, "plain or BN-statistics epilogue");
  static_assert(KS % PD == 0 && PD >= 1 && PD <= KS, "step sets tile the K chunks");
  constexpr int BM = 128, BN = 64, NT = 256, WM = 2, WN = 2;
  constexpr int WNB = BN / WN, FNW = WNB / 16;
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;
  constexpr int A_ELEMS = BM * BK, Y_ELEMS = BM * BN, W_ELEMS = KS * BK * BN;
  constexpr int CPA = A_ELEMS / 8 / NT, CPY = Y_ELEMS / 8 / NT, CPW = W_ELEMS / 8 / NT;
  constexpr int RSTEP = NT / 8;
  constexpr int K = KS * BK, N = BN, STEPS = KS, K8 = K >> 3;
  constexpr bool BNS = EPI == EPI_BF16_BN;
  constexpr int IT = BM * BN / 8 / NT;  // epilogue rows per thread (one 8-column group each)
  constexpr int PARTS = NT / (BN / 8);
  using EL = EpiLayout<BN>;
  static_assert(BM * EL::LD <= A_ELEMS + Y_ELEMS && 2 * PARTS * BN * 2 <= A_ELEMS + Y_ELEMS,
                "epilogue staging fits As + Ys");
  // LDS: As (dz chunk) | Ys (y tile) | Ws (all of W, 64-row chunks) | coefficients
  __shared__ __attribute__((aligned(16))) short smem[A_ELEMS + Y_ELEMS + W_ELEMS + 3 * K * 2];
  short* const As = smem;
  short* const Ys = smem + A_ELEMS;
  short* const Ws = Ys + Y_ELEMS;
  float* const Cf = reinterpret_cast<float*>(Ws + W_ELEMS);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_m = (P.M + BM - 1) / BM;
  const int t_beg = blockIdx.x * tiles_per_block;
  int t_end = t_beg + tiles_per_block;
  if (t_end > tiles_m) t_end = tiles_m;
  const int arow = tid >> 3, c8 = tid & 7;
  const int ecol = (tid % (BN / 8)) * 8;  // the epilogue's 8-column group

#pragma unroll
  for (int i = 0; i < CPW; ++i) {  // W [K][N] -> one swizzled 64 x 64 image per K chunk
    const int c = tid + i * NT, kr = c / (BN / 8), lc = c % (BN / 8);
    const int lr = kr % BK;
    const s8v v = *reinterpret_cast<const s8v*>(P.B + (long)kr * P.ldb + 8 * lc);
    *reinterpret_cast<s8v*>(Ws + (kr / BK) * (BK * BN) + lr * BN + ((lc ^ nc_swz<BN>(lr)) << 3)) = v;
  }
  for (int i = tid; i < 3 * K; i += NT) {
    const int q = i / K, k = i - q * K;
    Cf[i] = (q == 0 ? X.c0 : (q == 1 ? X.c1 : X.c2))[k];
  }

  // operand windows over the workgroup's whole tile range [t_beg, t_end) (rows past M or past
  // the range read zeros)
  const long r0 = (long)t_beg * BM;
  long rl = (long)P.M - r0;
  if (rl > (long)(t_end - t_beg) * BM) rl = (long)(t_end - t_beg) * BM;
  const auto r0s = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(X.src0 + r0 * P.lda), (short)0,
                                                     (int)buf_span(rl * P.lda * 2), 0x00020000);
  const auto r1s = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(X.src1 + r0 * P.lda), (short)0,
                                                     (int)buf_span(rl * P.lda * 2), 0x00020000);
  const auto rms = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(X.mask_in ? X.mask_in + r0 * K8 : reinterpret_cast<const uint8_t*>(ca_zero16)), (short)0,
      X.mask_in ? (int)buf_span(rl * K8) : 0, 0x00020000);
  const auto rys = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(Y + r0 * ldy), (short)0,
                                                     (int)buf_span(rl * ldy * 2), 0x00020000);
  const auto rzs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(BNS ? P.bnz + r0 * P.ldc : ca_zero16), (short)0, BNS ? (int)buf_span(rl * P.ldc * 2) : 0,
      0x00020000);
  const bool has_bnmask = BNS && P.bnmask != nullptr;
  const auto rbm = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(has_bnmask ? P.bnmask + r0 * (N / 8) : reinterpret_cast<const uint8_t*>(ca_zero16)),
      (short)0, has_bnmask ? (int)buf_span(rl * (N / 8)) : 0, 0x00020000);

  f4v accw[STEPS][2][FNW];
#pragma unroll
  for (int c = 0; c < STEPS; ++c)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < FNW; ++j) accw[c][i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  s8v a0[PD][CPA], a1[PD][CPA], yv[CPY], zp[BNS ? IT : 1];
  uint32_t mb[PD][CPA], mk[BNS ? IT : 1];

  auto load_a = [&](int p, int lt, int t) {  // set p <- dz sources of K chunk t of range tile lt
    const int k = t * BK + 8 * c8;
#pragma unroll
    for (int i = 0; i < CPA; ++i) {
      const int row = lt * BM + arow + i * RSTEP;
      const uint32_t off = (uint32_t)(((long)row * P.lda + k) * 2);
      a0[p][i] = __builtin_bit_cast(s8v, __builtin_amdgcn_raw_buffer_load_b128(r0s, (int)off, 0, 0));
      a1[p][i] = __builtin_bit_cast(s8v, __builtin_amdgcn_raw_buffer_load_b128(r1s, (int)off, 0, 0));
      mb[p][i] = __builtin_amdgcn_raw_buffer_load_b8(rms, row * K8 + (k >> 3), 0, 0);
    }
  };
  auto load_y = [&](int lt) {
#pragma unroll
    for (int i = 0; i < CPY; ++i) {
      const int c = tid + i * NT, lr = c / (BN / 8), lc = c % (BN / 8);
      yv[i] = __builtin_bit_cast(
          s8v, __builtin_amdgcn_raw_buffer_load_b128(rys, (int)(((long)(lt * BM + lr) * ldy + 8 * lc) * 2), 0, 0));
    }
  };
  auto load_epi = [&](int lt) {  // z and ReLU mask of the BN that consumes dx, this thread's IT rows
#pragma unroll
    for (int u = 0; u < IT; ++u) {
      const int row = lt * BM + (tid + u * NT) / (BN / 8);
      zp[u] = __builtin_bit_cast(
          s8v, __builtin_amdgcn_raw_buffer_load_b128(rzs, (int)(((long)row * P.ldc + ecol) * 2), 0, 0));
      mk[u] = has_bnmask ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rbm, row * (N / 8) + (ecol >> 3), 0, 0)
                         : 0xffu;
    }
  };
  auto store_a = [&](int p, int t) {  // dz = A*(dy*relu') + B*z + D  (bn_bwd_apply_kernel)
    const int k = t * BK + 8 * c8;
    f4v cf[3][2];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      cf[q][0] = *reinterpret_cast<const f4v*>(Cf + q * K + k);
      cf[q][1] = *reinterpret_cast<const f4v*>(Cf + q * K + k + 4);
    }
#pragma unroll
    for (int i = 0; i < CPA; ++i) {
      const int row = arow + i * RSTEP;
      s8v o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float d = bf2f((bf16_t)a0[p][i][j]);
        if (X.mask_in) d = ((mb[p][i] >> j) & 1u) ? d : 0.f;
        o[j] = (short)f2bf(bn_bwd_affine(cf[0][j >> 2][j & 3], d, cf[1][j >> 2][j & 3], bf2f((bf16_t)a1[p][i][j]),
                                         cf[2][j >> 2][j & 3]));
      }
      *reinterpret_cast<s8v*>(As + row * BK + ((c8 ^ (row & 7)) << 3)) = o;
    }
  };
  auto store_y = [&]() {
#pragma unroll
    for (int i = 0; i < CPY; ++i) {
      const int c = tid + i * NT, lr = c / (BN / 8), lc = c % (BN / 8);
      *reinterpret_cast<s8v*>(Ys + lr * BN + ((lc ^ nc_swz<BN>(lr)) << 3)) = yv[i];
    }
  };

  load_y(0);
#pragma unroll
  for (int p = 0; p < PD; ++p) load_a(p, 0, p);
  __syncthreads();  // W and the coefficient table are in LDS

  bf16_t* Cg = reinterpret_cast<bf16_t*>(P.C);
#pragma unroll 1
  for (int tm = t_beg; tm < t_end; ++tm) {
    const int lt = tm - t_beg, m0 = tm * BM;
    f4v acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
      store_a(s % PD, s);
      if (s == 0) store_y();
      // PD == KS: every refill is the next tile's, so this tile's epilogue operands go first
      if (BNS && PD == STEPS && s == 0) load_epi(lt);
      const int s2 = s + PD;  // refill the set just consumed
      if (s2 < STEPS) {
        load_a(s2 % PD, lt, s2);
        if (BNS && s2 == STEPS - 1) load_epi(lt);
      } else {
        if (s2 == STEPS) load_y(lt + 1);
        load_a(s2 % PD, lt + 1, s2 - STEPS);
      }
      lgkm_wait0();
      bar256();
      const short* Bs = Ws + s * (BK * BN);
#pragma unroll 1
      for (int kk = 0; kk < BK; kk += 32) {
        bf16x8 af[FM], bfr[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) af[i] = read_frag_sw<BM, true>(As, wm * (BM / WM) + i * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < FN; ++j) bfr[j] = read_frag_sw<BN, false>(Bs, wn * (BN / WN) + j * 16, kk, lane);
        mfma_acc<FM, FN>(acc, af, bfr);
      }
#pragma unroll 1
      for (int mk0 = 0; mk0 < BM; mk0 += 32) {
        bf16x8 dzt[2], yf[FNW];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
          const int mr = mk0 + 8 * g + q;
          const int lc = ((wm * 32 + i * 16) >> 3) + (pp >> 1);
          const int sub = 4 * (pp & 1);
          const short* b0 = As + mr * BK + ((lc ^ (mr & 7)) << 3) + sub;
          const short* b1 = As + (mr + 4) * BK + ((lc ^ ((mr + 4) & 7)) << 3) + sub;
          s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(b0));
          s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(b1));
          dzt[i] = __builtin_bit_cast(bf16x8, s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
        }
#pragma unroll
        for (int j = 0; j < FNW; ++j) yf[j] = read_frag_sw<BN, false>(Ys, wn * WNB + j * 16, mk0, lane);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < FNW; ++j)
            accw[s][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(yf[j], dzt[i], accw[s][i][j], 0, 0, 0);
      }
      lgkm_wait0();
      bar256();
    }

    // epilogue (gemm_epilogue, EPI_BF16 / EPI_BF16_BN at beta 0): C tile -> LDS (As + Ys) as bf16
    {
      short* Cs = As;
      const int rbase = wm * (BM / WM) + (lane & 15), cbase = wn * (BN / WN) + 4 * (lane >> 4);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          s4v pk;
#pragma unroll
          for (int r = 0; r < 4; ++r) pk[r] = (short)f2bf(acc[i][j][r]);
          *reinterpret_cast<s4v*>(Cs + EL::idx(rbase + i * 16, cbase + j * 16)) = pk;
        }
      __syncthreads();
      float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, bzsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      (void)bsum;
      (void)bzsum;
#pragma unroll
      for (int u = 0; u < IT; ++u) {
        const int row = (tid + u * NT) / (BN / 8), gm = m0 + row;
        if (gm >= P.M) continue;
        const s8v v = *reinterpret_cast<const s8v*>(Cs + EL::idx(row, ecol));
        *reinterpret_cast<s8v*>(Cg + (long)gm * P.ldc + ecol) = v;
        if constexpr (BNS) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float g = ((mk[u] >> j) & 1u) ? bf2f((bf16_t)v[j]) : 0.f;
            bsum[j] += g;
            bzsum[j] += g * bf2f((bf16_t)zp[u][j]);
          }
        }
      }
      if constexpr (BNS) {
        const int cg = tid % (BN / 8), part = tid / (BN / 8);
        __syncthreads();  // Cs consumed (sred aliases it)
        float* sred = reinterpret_cast<float*>(smem);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          sred[part * BN + cg * 8 + j] = bsum[j];
          sred[(PARTS + part) * BN + cg * 8 + j] = bzsum[j];
        }
        __syncthreads();
        for (int c = tid; c < BN; c += NT) {
          float ts = 0.f, tq = 0.f;
          for (int pp = 0; pp < PARTS; ++pp) {
            ts += sred[pp * BN + c];
            tq += sred[(PARTS + pp) * BN + c];
          }
          float* st = P.stats + (long)tm * 2 * P.N;
          st[c] = ts;
          st[P.N + c] = tq;
        }
      }
      __syncthreads();  // As / Ys free for the next tile's stores
    }
  }
  vm_wait<0>();  // the range's last refill reads nothing, but let it retire before the slab stores

  float* slab = ws + (long)blockIdx.x * K * N;
#pragma unroll
  for (int s = 0; s < STEPS; ++s)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < FNW; ++j) {
        const int k = s * BK + wm * 32 + i * 16 + (lane & 15);
        const int n = wn * WNB + j * 16 + 4 * (lane >> 4);
        *reinterpret_cast<f4v*>(slab + (long)k * N + n) = accw[s][i][j];
      }
}

}  // namespace ca
