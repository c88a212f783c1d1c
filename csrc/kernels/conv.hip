// Implicit-GEMM NHWC convolutions on MFMA (K2 in SURVEY.md 2.7): forward,
// input gradient (dgrad) and weight gradient (wgrad) of any KHxKW / stride /
// padding convolution with Cin, Cout multiples of 8 -- the whole of ResNet-50
// (7x7/2 stem on 8-channel-padded input, 3x3/1, 3x3/2, 1x1/2) runs here, so
// no convolution kernel is JIT-compiled at first use.
//
// GEMM views (weights stored [Cout][KH][KW][Cin]; k orders taps outer, channels inner):
//   fwd   : Y [m=(n,oh,ow)][co]      = sum_{k=(tap,ci)}  X[n, oh*s-p+kh, ow*s-p+kw, ci] * W[co][tap][ci]
//   dgrad : dX[m=(n,ih,iw)][ci]      = sum_{k=(tap,co)} dY[n, (ih+p-kh)/s, (iw+p-kw)/s, co] * W[co][tap][ci]
//                                      (terms with a non-integral or out-of-range output index are zero)
//   wgrad : dW[co][j=(tap,ci)]      = sum_{k=(n,oh,ow)} dY[k][co] * X[n, oh*s-p+kh, ow*s-p+kw, ci]
// Every operand chunk is 8 consecutive channels of one pixel (16 B), gathered
// per lane; the MFMA core (ca_mfma_core.h) does the rest.  wgrad is split-K
// over the N*OH*OW reduction with fp32 slabs.
#include <stdlib.h>
#include <string.h>

#include "ca_conv_halo.h"
#include "ca_conv_stem.h"
#include "ca_mfma_core.h"

namespace {
using namespace ca;

struct Pix {
  int n, y, x;
};
__device__ __forceinline__ Pix decode(uint32_t m, const FastDiv& dw, const FastDiv& dh) {
  const uint32_t t = fdiv(m, dw);
  const uint32_t x = m - t * dw.d;
  const uint32_t n = fdiv(t, dh);
  return Pix{(int)n, (int)(t - n * dh.d), (int)x};
}

// (tap, channel) of reduction index k over `C` channels per tap.  When C is a
// multiple of BK a K tile never straddles two taps, so the tap is uniform and
// derived from the tile start only.
__device__ __forceinline__ void tap_split(int k, int k0, int C, const FastDiv& dc, bool tile_in_tap, int& tap,
                                          int& c) {
  tap = (int)fdiv((uint32_t)(tile_in_tap ? k0 : k), dc);
  c = k - tap * C;
}

// A of forward: rows = output pixels, k = (tap, ci).  KC.
template <int R, int CPT, int NT>
struct ConvFwdA {
  static constexpr bool KC = true;
  const CoreParams& P;
  const bf16_t* nbase[CPT];
  int iy0[CPT], ix0[CPT], col[CPT];
  __device__ ConvFwdA(const CoreParams& p, bool, int r0, int tid) : P(p) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      int row, c;
      chunk_coords<R, true>(tid + i * NT, row, c);
      const int m = r0 + row;
      col[i] = c;
      if (m < P.M) {
        const Pix o = decode((uint32_t)m, P.div_ow, P.div_oh);
        nbase[i] = P.A + (long)o.n * P.H * P.W * P.Cin;
        iy0[i] = o.y * P.sh - P.ph;
        ix0[i] = o.x * P.sw - P.pw;
      } else {
        nbase[i] = P.A;
        iy0[i] = -(1 << 29);  // forces out-of-range
        ix0[i] = 0;
      }
    }
  }
  __device__ __forceinline__ s8v load(int i, int k0) const {
    const int k = k0 + col[i];
    if (k >= P.K) return zero8();
    int tap, ci;
    tap_split(k, k0, P.Cin, P.div_cin, P.cin_tile, tap, ci);
    const int kh = (int)fdiv((uint32_t)tap, P.div_kw), kw = tap - kh * P.KW;
    const int ih = iy0[i] + kh, iw = ix0[i] + kw;
    if ((unsigned)ih >= (unsigned)P.H || (unsigned)iw >= (unsigned)P.W) return zero8();
    return ld16(nbase[i] + ((long)ih * P.W + iw) * P.Cin + ci);
  }
};

// A of dgrad: rows = input pixels, k = (tap, co) over dY.  KC.
template <int R, int CPT, int NT>
struct ConvDgradA {
  static constexpr bool KC = true;
  const CoreParams& P;
  const bf16_t* nbase[CPT];
  int iy[CPT], ix[CPT], col[CPT];
  __device__ ConvDgradA(const CoreParams& p, bool, int r0, int tid) : P(p) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      int row, c;
      chunk_coords<R, true>(tid + i * NT, row, c);
      const int m = r0 + row;
      col[i] = c;
      if (m < P.M) {
        const Pix q = decode((uint32_t)m, P.div_w, P.div_h);
        nbase[i] = P.A + (long)q.n * P.OH * P.OW * P.Cout;
        iy[i] = q.y + P.ph;
        ix[i] = q.x + P.pw;
      } else {
        nbase[i] = P.A;
        iy[i] = -(1 << 29);
        ix[i] = 0;
      }
    }
  }
  __device__ __forceinline__ s8v load(int i, int k0) const {
    const int k = k0 + col[i];
    if (k >= P.K) return zero8();
    int tap, co;
    tap_split(k, k0, P.Cout, P.div_cout, P.cout_tile, tap, co);
    const int kh = (int)fdiv((uint32_t)tap, P.div_kw), kw = tap - kh * P.KW;
    int oy = iy[i] - kh, ox = ix[i] - kw;
    if (oy < 0 || ox < 0) return zero8();
    if (P.sh > 1) {
      if (oy % P.sh) return zero8();
      oy /= P.sh;
    }
    if (P.sw > 1) {
      if (ox % P.sw) return zero8();
      ox /= P.sw;
    }
    if (oy >= P.OH || ox >= P.OW) return zero8();
    return ld16(nbase[i] + ((long)oy * P.OW + ox) * P.Cout + co);
  }
};

// B of dgrad: B[k=(tap,co)][ci] = W[co][tap][ci]  (ci contiguous -> NC).
template <int R, int CPT, int NT>
struct ConvDgradB {
  static constexpr bool KC = false;
  const CoreParams& P;
  int row[CPT], ci[CPT];
  bool ok[CPT];
  __device__ ConvDgradB(const CoreParams& p, bool, int r0, int tid) : P(p) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      int r, c;
      chunk_coords<R, false>(tid + i * NT, r, c);
      row[i] = r;
      ci[i] = r0 + c;
      ok[i] = ci[i] < P.N;
    }
  }
  __device__ __forceinline__ s8v load(int i, int k0) const {
    const int k = k0 + row[i];
    if (!ok[i] || k >= P.K) return zero8();
    int tap, co;
    tap_split(k, k0, P.Cout, P.div_cout, P.cout_tile, tap, co);
    return ld16(P.B + ((long)co * (P.KH * P.KW) + tap) * P.Cin + ci[i]);
  }
};

// B of wgrad: B[k=(n,oh,ow)][j=(tap,ci)] = X[n, oh*s-p+kh, ow*s-p+kw, ci]  (NC).
template <int R, int CPT, int NT>
struct ConvWgradB {
  static constexpr bool KC = false;
  const CoreParams& P;
  int row[CPT], kh[CPT], kw[CPT], ci[CPT];
  bool ok[CPT];
  __device__ ConvWgradB(const CoreParams& p, bool, int r0, int tid) : P(p) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      int r, c;
      chunk_coords<R, false>(tid + i * NT, r, c);
      row[i] = r;
      const int j = r0 + c;
      ok[i] = j < P.N;
      int tap, cc;
      tap_split(ok[i] ? j : 0, 0, P.Cin, P.div_cin, false, tap, cc);
      const int h = (int)fdiv((uint32_t)tap, P.div_kw);
      kh[i] = h;
      kw[i] = tap - h * P.KW;
      ci[i] = cc;
    }
  }
  __device__ __forceinline__ s8v load(int i, int k0) const {
    const int k = k0 + row[i];
    if (!ok[i] || k >= P.K) return zero8();
    const Pix o = decode((uint32_t)k, P.div_ow, P.div_oh);
    const int ih = o.y * P.sh - P.ph + kh[i], iw = o.x * P.sw - P.pw + kw[i];
    if ((unsigned)ih >= (unsigned)P.H || (unsigned)iw >= (unsigned)P.W) return zero8();
    return ld16(P.B + (((long)o.n * P.H + ih) * P.W + iw) * P.Cin + ci[i]);
  }
};

// ---------------------------------------------------------------------------
// LDS-DMA (glds) versions of the gather loaders: they return the 16-B source
// address of each chunk (the zero page for padding / out-of-range taps) and
// follow the swizzled chunk order of mfma_gemm_glds (ca_mfma_core.h).  Row
// (pixel) state that differs per chunk is precomputed; the swizzled column
// slot is the same for every chunk of a thread.

template <int R, int CPT, int NT>
struct GConvFwdA {
  static constexpr bool KC = true;
  const CoreParams& P;
  const bf16_t* nbase[CPT];
  int iy0[CPT], ix0[CPT];
  int col;
  __device__ GConvFwdA(const CoreParams& p, bool, int r0, int tid) : P(p) {
    const int row_t = tid >> 3;
    col = ((tid & 7) ^ (row_t & 7)) << 3;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int m = r0 + row_t + i * (NT / 8);
      if (m < P.M) {
        const Pix o = decode((uint32_t)m, P.div_ow, P.div_oh);
        nbase[i] = P.A + (long)o.n * P.H * P.W * P.Cin;
        iy0[i] = o.y * P.sh - P.ph;
        ix0[i] = o.x * P.sw - P.pw;
      } else {
        nbase[i] = P.A;
        iy0[i] = -(1 << 29);
        ix0[i] = 0;
      }
    }
  }
  __device__ __forceinline__ const bf16_t* src(int i, int k0) const {
    const int k = k0 + col;
    if (k >= P.K) return ca_zero16;
    int tap, ci;
    tap_split(k, k0, P.Cin, P.div_cin, P.cin_tile, tap, ci);
    const int kh = (int)fdiv((uint32_t)tap, P.div_kw), kw = tap - kh * P.KW;
    const int ih = iy0[i] + kh, iw = ix0[i] + kw;
    if ((unsigned)ih >= (unsigned)P.H || (unsigned)iw >= (unsigned)P.W) return ca_zero16;
    return nbase[i] + ((long)ih * P.W + iw) * P.Cin + ci;
  }
};

template <int R, int CPT, int NT>
struct GConvDgradA {
  static constexpr bool KC = true;
  const CoreParams& P;
  const bf16_t* nbase[CPT];
  int iy[CPT], ix[CPT];
  int col;
  __device__ GConvDgradA(const CoreParams& p, bool, int r0, int tid) : P(p) {
    const int row_t = tid >> 3;
    col = ((tid & 7) ^ (row_t & 7)) << 3;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int m = r0 + row_t + i * (NT / 8);
      if (m < P.M) {
        const Pix q = decode((uint32_t)m, P.div_w, P.div_h);
        nbase[i] = P.A + (long)q.n * P.OH * P.OW * P.Cout;
        iy[i] = q.y + P.ph;
        ix[i] = q.x + P.pw;
      } else {
        nbase[i] = P.A;
        iy[i] = -(1 << 29);
        ix[i] = 0;
      }
    }
  }
  __device__ __forceinline__ const bf16_t* src(int i, int k0) const {
    const int k = k0 + col;
    if (k >= P.K) return ca_zero16;
    int tap, co;
    tap_split(k, k0, P.Cout, P.div_cout, P.cout_tile, tap, co);
    const int kh = (int)fdiv((uint32_t)tap, P.div_kw), kw = tap - kh * P.KW;
    int oy = iy[i] - kh, ox = ix[i] - kw;
    if (oy < 0 || ox < 0) return ca_zero16;
    if (P.sh > 1) {
      if (oy % P.sh) return ca_zero16;
      oy /= P.sh;
    }
    if (P.sw > 1) {
      if (ox % P.sw) return ca_zero16;
      ox /= P.sw;
    }
    if (oy >= P.OH || ox >= P.OW) return ca_zero16;
    return nbase[i] + ((long)oy * P.OW + ox) * P.Cout + co;
  }
};

// B of dgrad: B[k=(tap,co)][ci] = W[co][tap][ci] (NC).
template <int R, int CPT, int NT>
struct GConvDgradB {
  static constexpr bool KC = false;
  const CoreParams& P;
  int krow0, ci;
  __device__ GConvDgradB(const CoreParams& p, bool, int r0, int tid) : P(p) {
    constexpr int CPR = R / 8;
    const int k = tid / CPR, pc = tid % CPR;
    int n = r0 + ((pc ^ nc_swz<R>(k)) << 3);
    if (n > P.N - 8) n = P.N - 8;
    ci = n;
    krow0 = k;
  }
  __device__ __forceinline__ const bf16_t* src(int i, int k0) const {
    const int k = k0 + krow0 + i * (NT * 8 / R);
    if (k >= P.K) return ca_zero16;
    int tap, co;
    tap_split(k, k0, P.Cout, P.div_cout, P.cout_tile, tap, co);
    return P.B + ((long)co * (P.KH * P.KW) + tap) * P.Cin + ci;
  }
};

// B of wgrad: B[k=(n,oh,ow)][j=(tap,ci)] = X[n, oh*s-p+kh, ow*s-p+kw, ci] (NC).
template <int R, int CPT, int NT>
struct GConvWgradB {
  static constexpr bool KC = false;
  const CoreParams& P;
  int krow0, kh, kw, ci;
  __device__ GConvWgradB(const CoreParams& p, bool, int r0, int tid) : P(p) {
    constexpr int CPR = R / 8;
    const int k = tid / CPR, pc = tid % CPR;
    int j = r0 + ((pc ^ nc_swz<R>(k)) << 3);
    if (j > P.N - 8) j = P.N - 8;
    int tap, cc;
    tap_split(j, 0, P.Cin, P.div_cin, false, tap, cc);
    kh = (int)fdiv((uint32_t)tap, P.div_kw);
    kw = tap - kh * P.KW;
    ci = cc;
    krow0 = k;
  }
  __device__ __forceinline__ const bf16_t* src(int i, int k0) const {
    const int k = k0 + krow0 + i * (NT * 8 / R);
    if (k >= P.K) return ca_zero16;
    const Pix o = decode((uint32_t)k, P.div_ow, P.div_oh);
    const int ih = o.y * P.sh - P.ph + kh, iw = o.x * P.sw - P.pw + kw;
    if ((unsigned)ih >= (unsigned)P.H || (unsigned)iw >= (unsigned)P.W) return ca_zero16;
    return P.B + (((long)o.n * P.H + ih) * P.W + iw) * P.Cin + ci;
  }
};

// ---- tap-mask gather loaders (K tile = one tap x 64 channels) ----------------
// When the gathered operand's channel count is a multiple of BK, a K tile is one
// filter tap and one 64-channel slice, so the tap (kh, kw) and the channel offset are
// wave-uniform: the per-tile address work moves to the scalar unit.  Each chunk keeps a
// 64-bit pointer to its centre pixel and a bitmask of the taps that land inside the image
// (computed once); per K tile a lane only tests one bit and adds the uniform tap offset,
// selecting the zero page without a branch.  The general loaders above spend ~25 VALU
// and two divergent branches per chunk per K tile, which on the 64-channel layers costs
// more issue time than the tile's 16 MFMAs.  Needs KH*KW (taps per class) <= 32.
struct TapOff {
  int tap;  // filter tap (kh * KW + kw) of the K tile
  int c;    // channel offset of the K tile within the tap
  long sp;  // (kh * pitch + kw) * C: spatial part of the element offset
};
__device__ __forceinline__ TapOff tap_offset(int k0, const FastDiv& dc, int C, const FastDiv& dkw, int KW, int pitch) {
  TapOff t;
  t.tap = (int)fdiv((uint32_t)k0, dc);
  t.c = k0 - t.tap * C;
  const int kh = (int)fdiv((uint32_t)t.tap, dkw), kw = t.tap - kh * KW;
  t.sp = ((long)kh * pitch + kw) * C;
  return t;
}

// forward A: X[n, oy*s - p + kh, ox*s - p + kw, c]; Cin % BK == 0.
template <int R, int CPT, int NT>
struct GConvFwdAT {
  static constexpr bool KC = true, BUF = true;
  const CoreParams& P;
  const bf16_t* sbase;  // &X[n0] (image of the tile's first row)
  uint32_t nrec;
  int32_t cofs[CPT];  // byte offset of X[n, oy*s - p, ox*s - p, col] from sbase (may be < 0)
  uint32_t vm[CPT];   // bit kh*KW + kw: that tap is inside the image
  __device__ GConvFwdAT(const CoreParams& p, bool, int r0, int tid) : P(p) {
    const int row_t = tid >> 3;
    const int col = ((tid & 7) ^ (row_t & 7)) << 3;
    const long img = (long)P.H * P.W * P.Cin;
    const int n0 = (int)fdiv(fdiv((uint32_t)r0, P.div_ow), P.div_oh);
    sbase = P.A + n0 * img;
    nrec = buf_span((P.Nb - n0) * img * 2);
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int m = r0 + row_t + i * (NT / 8);
      uint32_t mask = 0;
      long off = 0;
      if (m < P.M) {
        const Pix o = decode((uint32_t)m, P.div_ow, P.div_oh);
        const int iy0 = o.y * P.sh - P.ph, ix0 = o.x * P.sw - P.pw;
        off = (((long)(o.n - n0) * P.H + iy0) * P.W + ix0) * P.Cin + col;
        for (int kh = 0; kh < P.KH; ++kh) {
          if ((unsigned)(iy0 + kh) >= (unsigned)P.H) continue;
          for (int kw = 0; kw < P.KW; ++kw)
            if ((unsigned)(ix0 + kw) < (unsigned)P.W) mask |= 1u << (kh * P.KW + kw);
        }
      }
      cofs[i] = (int32_t)(off * 2);
      vm[i] = mask;
    }
  }
  __device__ __forceinline__ uint32_t off(int i, int k0) const {
    const TapOff t = tap_offset(k0, P.div_cin, P.Cin, P.div_kw, P.KW, P.W);
    const uint32_t o = (uint32_t)cofs[i] + (uint32_t)((t.sp + t.c) * 2);
    return ((vm[i] >> t.tap) & 1u) ? o : nrec;
  }
};

// forward A of a stride-1, unpadded convolution whose kernel row spans exactly one K tile
// (KW * Cin == BK): the space-to-depth ResNet stem, 4x4 over 16 channels.  K tile kh of
// output pixel (n, oy, ox) is the CONTIGUOUS 128-B run X[n, oy + kh, ox .. ox + KW - 1, :],
// so a chunk's address is its row base plus kh whole input rows -- no per-tile tap decode
// (the general GConvFwdA loader re-derives tap and channel for every chunk and K tile).
template <int R, int CPT, int NT>
struct GConvRowA {
  static constexpr bool KC = true, BUF = true;
  const CoreParams& P;
  const bf16_t* sbase;  // &X[n0]
  uint32_t nrec;
  uint32_t rofs[CPT];   // byte offset of X[n, oy, ox, col] from sbase; nrec for rows past M
  uint32_t rowb;        // bytes of one input row (W * Cin * 2)
  __device__ GConvRowA(const CoreParams& p, bool, int r0, int tid) : P(p) {
    const int row_t = tid >> 3;
    const int col = ((tid & 7) ^ (row_t & 7)) << 3;
    const long img = (long)P.H * P.W * P.Cin;
    const int n0 = (int)fdiv(fdiv((uint32_t)r0, P.div_ow), P.div_oh);
    sbase = P.A + n0 * img;
    nrec = buf_span((P.Nb - n0) * img * 2);
    rowb = (uint32_t)(P.W * P.Cin * 2);
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int m = r0 + row_t + i * (NT / 8);
      uint32_t o = nrec;
      if (m < P.M) {
        const Pix q = decode((uint32_t)m, P.div_ow, P.div_oh);
        o = (uint32_t)(((((long)(q.n - n0) * P.H + q.y) * P.W + q.x) * P.Cin + col) * 2);
      }
      rofs[i] = o;
    }
  }
  __device__ __forceinline__ uint32_t off(int i, int k0) const {
    return rofs[i] >= nrec ? nrec : rofs[i] + (uint32_t)(k0 / BK) * rowb;
  }
};

// stride-1 dgrad A: dY[n, iy + p - kh, ix + p - kw, co]; Cout % BK == 0.
template <int R, int CPT, int NT>
struct GConvDgradAT {
  static constexpr bool KC = true, BUF = true;
  const CoreParams& P;
  const bf16_t* sbase;  // &dY[n0]
  uint32_t nrec;
  int32_t cofs[CPT];  // byte offset of dY[n, iy + p, ix + p, col] from sbase
  uint32_t vm[CPT];
  __device__ GConvDgradAT(const CoreParams& p, bool, int r0, int tid) : P(p) {
    const int row_t = tid >> 3;
    const int col = ((tid & 7) ^ (row_t & 7)) << 3;
    const long img = (long)P.OH * P.OW * P.Cout;
    const int n0 = (int)fdiv(fdiv((uint32_t)r0, P.div_w), P.div_h);
    sbase = P.A + n0 * img;
    nrec = buf_span((P.Nb - n0) * img * 2);
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int m = r0 + row_t + i * (NT / 8);
      uint32_t mask = 0;
      long off = 0;
      if (m < P.M) {
        const Pix q = decode((uint32_t)m, P.div_w, P.div_h);
        const int oy0 = q.y + P.ph, ox0 = q.x + P.pw;
        off = (((long)(q.n - n0) * P.OH + oy0) * P.OW + ox0) * P.Cout + col;
        for (int kh = 0; kh < P.KH; ++kh) {
          if ((unsigned)(oy0 - kh) >= (unsigned)P.OH) continue;
          for (int kw = 0; kw < P.KW; ++kw)
            if ((unsigned)(ox0 - kw) < (unsigned)P.OW) mask |= 1u << (kh * P.KW + kw);
        }
      }
      cofs[i] = (int32_t)(off * 2);
      vm[i] = mask;
    }
  }
  __device__ __forceinline__ uint32_t off(int i, int k0) const {
    const TapOff t = tap_offset(k0, P.div_cout, P.Cout, P.div_kw, P.KW, P.OW);
    const uint32_t o = (uint32_t)cofs[i] + (uint32_t)((t.c - t.sp) * 2);  // the gather walks back by the tap
    return ((vm[i] >> t.tap) & 1u) ? o : nrec;
  }
};

// Branch-free form of GConvWgradB: one pixel decode per chunk, the validity test folded
// into sel_src.  For a stride-1 "same" convolution (OH == H, OW == W) the source address is
// linear in the pixel index: X + (k + (kh - p) * W + (kw - p)) * Cin + ci.
template <int R, int CPT, int NT>
struct GConvWgradBT {
  static constexpr bool KC = false;
  const CoreParams& P;
  const bf16_t* tbase;  // X + ((kh - ph) * W + (kw - pw)) * Cin + ci
  int krow0, dh, dw, ci;
  bool lin;
  __device__ GConvWgradBT(const CoreParams& p, bool, int r0, int tid) : P(p) {
    constexpr int CPR = R / 8;
    const int k = tid / CPR, pc = tid % CPR;
    int j = r0 + ((pc ^ nc_swz<R>(k)) << 3);
    if (j > P.N - 8) j = P.N - 8;
    int tap, cc;
    tap_split(j, 0, P.Cin, P.div_cin, false, tap, cc);
    const int kh = (int)fdiv((uint32_t)tap, P.div_kw);
    dh = kh - P.ph;
    dw = tap - kh * P.KW - P.pw;
    ci = cc;
    krow0 = k;
    tbase = P.B + ((long)dh * P.W + dw) * P.Cin + ci;
    lin = P.sh == 1 && P.sw == 1 && P.OH == P.H && P.OW == P.W;
  }
  __device__ __forceinline__ const bf16_t* src(int i, int k0) const {
    const int k = k0 + krow0 + i * (NT * 8 / R);
    const Pix o = decode((uint32_t)k, P.div_ow, P.div_oh);
    const int ih = o.y * P.sh + dh, iw = o.x * P.sw + dw;
    const bool ok = k < P.K && (unsigned)ih < (unsigned)P.H && (unsigned)iw < (unsigned)P.W;
    const bf16_t* a = lin ? tbase + (long)k * P.Cin : P.B + (((long)o.n * P.H + ih) * P.W + iw) * P.Cin + ci;
    return sel_src(ok, a);
  }
};

// dgrad B with Cout % BK == 0: W[co][tap][ci], co = c0 + krow (c0, tap uniform per K tile).
template <int R, int CPT, int NT>
struct GConvDgradBT {
  static constexpr bool KC = false, BUF = true;
  static constexpr int KSTEP = NT * 8 / R;
  const CoreParams& P;
  const bf16_t* sbase;  // W
  uint32_t nrec;
  uint32_t wofs;  // byte offset of W[krow0][0][ci]
  int krow0;
  __device__ GConvDgradBT(const CoreParams& p, bool, int r0, int tid) : P(p) {
    constexpr int CPR = R / 8;
    const int k = tid / CPR, pc = tid % CPR;
    int n = r0 + ((pc ^ nc_swz<R>(k)) << 3);
    if (n > P.N - 8) n = P.N - 8;
    krow0 = k;
    sbase = P.B;
    nrec = buf_span((long)P.Cout * P.KH * P.KW * P.Cin * 2);
    wofs = (uint32_t)((n + (long)k * (P.KH * P.KW) * P.Cin) * 2);
  }
  __device__ __forceinline__ uint32_t off(int i, int k0) const {
    const int tap = (int)fdiv((uint32_t)k0, P.div_cout), c0 = k0 - tap * P.Cout;
    const uint32_t o = wofs + (uint32_t)((((long)(c0 + i * KSTEP) * (P.KH * P.KW) + tap) * P.Cin) * 2);
    return (k0 + krow0 + i * KSTEP < P.K) ? o : nrec;
  }
};

// Weight-gradient B walked incrementally: each chunk keeps its pixel (oy, ox) and source
// pointer and steps them BK pixels per K tile with uniform deltas (no per-tile division or
// 64-bit multiply).  One row carry and one image carry per step are enough when
// OH * OW >= 2 * BK (host-checked); smaller maps use GConvWgradBT.
template <int R, int CPT, int NT>
struct GConvWgradBI {
  static constexpr bool KC = false, BUF = true;
  static constexpr int KSTEP = NT * 8 / R;
  const CoreParams& P;
  const bf16_t* sbase;  // &X[n0]: image of the block's first pixel (split-K start)
  uint32_t nrec;
  uint32_t ofs[CPT];    // byte offset of X[n, oy*s + dh, ox*s + dw, ci] for the chunk's current pixel
  int oy[CPT], ox[CPT];
  int krow0, dh, dw;
  uint32_t dpa, dcx, dcy;  // byte steps: per tile, extra on a row carry, extra on an image carry
  int dxa, dya;
  __device__ GConvWgradBI(const CoreParams& p, bool, int r0, int tid) : P(p) {
    constexpr int CPR = R / 8;
    const int k = tid / CPR, pc = tid % CPR;
    int j = r0 + ((pc ^ nc_swz<R>(k)) << 3);
    if (j > P.N - 8) j = P.N - 8;
    int tap, ci;
    tap_split(j, 0, P.Cin, P.div_cin, false, tap, ci);
    const int kh = (int)fdiv((uint32_t)tap, P.div_kw);
    dh = kh - P.ph;
    dw = tap - kh * P.KW - P.pw;
    krow0 = k;
    dya = BK / P.OW;
    dxa = BK - dya * P.OW;
    const long rowp = (long)P.sh * P.W * P.Cin, colp = (long)P.sw * P.Cin, img = (long)P.H * P.W * P.Cin;
    dpa = (uint32_t)((dya * rowp + dxa * colp) * 2);
    dcx = (uint32_t)((rowp - (long)P.OW * colp) * 2);
    dcy = (uint32_t)((img - (long)P.OH * rowp) * 2);
    const int kbeg = blk_split(P) * P.k_per_split;
    const int n0 = (int)fdiv(fdiv((uint32_t)kbeg, P.div_ow), P.div_oh);
    sbase = P.B + n0 * img;
    nrec = buf_span((P.Nb - n0) * img * 2);
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const Pix o = decode((uint32_t)(kbeg + k + i * KSTEP), P.div_ow, P.div_oh);
      oy[i] = o.y;
      ox[i] = o.x;
      ofs[i] = (uint32_t)(((((long)(o.n - n0) * P.H + o.y * P.sh + dh) * P.W + o.x * P.sw + dw) * P.Cin + ci) * 2);
    }
  }
  __device__ __forceinline__ uint32_t off(int i, int k0) const {
    const int ih = __umul24(oy[i], P.sh) + dh, iw = __umul24(ox[i], P.sw) + dw;
    const bool ok = (k0 + krow0 + i * KSTEP < P.K) & ((unsigned)ih < (unsigned)P.H) & ((unsigned)iw < (unsigned)P.W);
    return ok ? ofs[i] : nrec;
  }
  __device__ __forceinline__ void advance() {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      int x = ox[i] + dxa, y = oy[i] + dya;
      uint32_t d = dpa;
      if (x >= P.OW) {
        x -= P.OW;
        y += 1;
        d += dcx;
      }
      if (y >= P.OH) {
        y -= P.OH;
        d += dcy;
      }
      ox[i] = x;
      oy[i] = y;
      ofs[i] += d;
    }
  }
};

// ---- strided dgrad by output-parity class (sub-pixel decomposition) ----------
// For stride s the input pixels with (iy % s, ix % s) = (py, px) only receive
// taps kh = kh0 + s*th (kh0 = (py + ph) % s), kw likewise, from dY row
// oy = qy + dy0 - th.  One GEMM per class: M = N*Hq*Wq, K = nh*nw*Cout -- no
// MFMA work on the (s^2-1)/s^2 structurally-zero products.

// A: rows = class pixels (n, qy, qx); k = (t = th*nw + tw, co) over dY.  KC.
template <int R, int CPT, int NT>
struct GConvDgradSA {
  static constexpr bool KC = true;
  const CoreParams& P;
  const bf16_t* nbase[CPT];
  int qy[CPT], qx[CPT];
  int col;
  __device__ GConvDgradSA(const CoreParams& p, bool, int r0, int tid) : P(p) {
    const int row_t = tid >> 3;
    col = ((tid & 7) ^ (row_t & 7)) << 3;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int m = r0 + row_t + i * (NT / 8);
      if (m < P.M) {
        const Pix q = decode((uint32_t)m, P.div_wq, P.div_hq);
        nbase[i] = P.A + (long)q.n * P.OH * P.OW * P.Cout;
        qy[i] = q.y + P.dg_dy0;
        qx[i] = q.x + P.dg_dx0;
      } else {
        nbase[i] = P.A;
        qy[i] = -(1 << 29);
        qx[i] = 0;
      }
    }
  }
  __device__ __forceinline__ const bf16_t* src(int i, int k0) const {
    const int k = k0 + col;
    if (k >= P.K) return ca_zero16;
    int t, co;
    tap_split(k, k0, P.Cout, P.div_cout, P.cout_tile, t, co);
    const int th = (int)fdiv((uint32_t)t, P.div_nw), tw = t - th * P.dg_nw;
    const int oy = qy[i] - th, ox = qx[i] - tw;
    if ((unsigned)oy >= (unsigned)P.OH || (unsigned)ox >= (unsigned)P.OW) return ca_zero16;
    return nbase[i] + ((long)oy * P.OW + ox) * P.Cout + co;
  }
};

// tap-mask form of GConvDgradSA (Cout % BK == 0, nh*nw <= 32): dY[n, qy + dy0 - th, qx + dx0 - tw, co].
template <int R, int CPT, int NT>
struct GConvDgradSAT {
  static constexpr bool KC = true, BUF = true;
  const CoreParams& P;
  const bf16_t* sbase;  // &dY[n0]
  uint32_t nrec;
  int32_t cofs[CPT];  // byte offset of dY[n, qy + dy0, qx + dx0, col] from sbase
  uint32_t vm[CPT];   // bit th*nw + tw
  __device__ GConvDgradSAT(const CoreParams& p, bool, int r0, int tid) : P(p) {
    const int row_t = tid >> 3;
    const int col = ((tid & 7) ^ (row_t & 7)) << 3;
    const long img = (long)P.OH * P.OW * P.Cout;
    const int n0 = (int)fdiv(fdiv((uint32_t)r0, P.div_wq), P.div_hq);
    sbase = P.A + n0 * img;
    nrec = buf_span((P.Nb - n0) * img * 2);
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int m = r0 + row_t + i * (NT / 8);
      uint32_t mask = 0;
      long off = 0;
      if (m < P.M) {
        const Pix q = decode((uint32_t)m, P.div_wq, P.div_hq);
        const int oy0 = q.y + P.dg_dy0, ox0 = q.x + P.dg_dx0;
        off = (((long)(q.n - n0) * P.OH + oy0) * P.OW + ox0) * P.Cout + col;
        for (int th = 0; th < P.dg_nh; ++th) {
          if ((unsigned)(oy0 - th) >= (unsigned)P.OH) continue;
          for (int tw = 0; tw < P.dg_nw; ++tw)
            if ((unsigned)(ox0 - tw) < (unsigned)P.OW) mask |= 1u << (th * P.dg_nw + tw);
        }
      }
      cofs[i] = (int32_t)(off * 2);
      vm[i] = mask;
    }
  }
  __device__ __forceinline__ uint32_t off(int i, int k0) const {
    const TapOff t = tap_offset(k0, P.div_cout, P.Cout, P.div_nw, P.dg_nw, P.OW);
    const uint32_t o = (uint32_t)cofs[i] + (uint32_t)((t.c - t.sp) * 2);
    return ((vm[i] >> t.tap) & 1u) ? o : nrec;
  }
};

// B: B[k=(t,co)][ci] = W[co][kh0 + s*th][kw0 + s*tw][ci]  (NC).
template <int R, int CPT, int NT>
struct GConvDgradSB {
  static constexpr bool KC = false;
  const CoreParams& P;
  int krow0, ci;
  __device__ GConvDgradSB(const CoreParams& p, bool, int r0, int tid) : P(p) {
    constexpr int CPR = R / 8;
    const int k = tid / CPR, pc = tid % CPR;
    int n = r0 + ((pc ^ nc_swz<R>(k)) << 3);
    if (n > P.N - 8) n = P.N - 8;
    ci = n;
    krow0 = k;
  }
  __device__ __forceinline__ const bf16_t* src(int i, int k0) const {
    const int k = k0 + krow0 + i * (NT * 8 / R);
    if (k >= P.K) return ca_zero16;
    int t, co;
    tap_split(k, k0, P.Cout, P.div_cout, P.cout_tile, t, co);
    const int th = (int)fdiv((uint32_t)t, P.div_nw), tw = t - th * P.dg_nw;
    const int kh = P.dg_kh0 + P.sh * th, kw = P.dg_kw0 + P.sw * tw;
    return P.B + ((long)co * (P.KH * P.KW) + kh * P.KW + kw) * P.Cin + ci;
  }
};

// class dgrad B with Cout % BK == 0: W[co][kh0 + s*th][kw0 + s*tw][ci], (t, c0) uniform per K tile.
template <int R, int CPT, int NT>
struct GConvDgradSBT {
  static constexpr bool KC = false, BUF = true;
  static constexpr int KSTEP = NT * 8 / R;
  const CoreParams& P;
  const bf16_t* sbase;
  uint32_t nrec;
  uint32_t wofs;
  int krow0;
  __device__ GConvDgradSBT(const CoreParams& p, bool, int r0, int tid) : P(p) {
    constexpr int CPR = R / 8;
    const int k = tid / CPR, pc = tid % CPR;
    int n = r0 + ((pc ^ nc_swz<R>(k)) << 3);
    if (n > P.N - 8) n = P.N - 8;
    krow0 = k;
    sbase = P.B;
    nrec = buf_span((long)P.Cout * P.KH * P.KW * P.Cin * 2);
    wofs = (uint32_t)((n + (long)k * (P.KH * P.KW) * P.Cin) * 2);
  }
  __device__ __forceinline__ uint32_t off(int i, int k0) const {
    const int t = (int)fdiv((uint32_t)k0, P.div_cout), c0 = k0 - t * P.Cout;
    const int th = (int)fdiv((uint32_t)t, P.div_nw), tw = t - th * P.dg_nw;
    const int kh = P.dg_kh0 + P.sh * th, kw = P.dg_kw0 + P.sw * tw;
    const uint32_t o = wofs + (uint32_t)((((long)(c0 + i * KSTEP) * (P.KH * P.KW) + kh * P.KW + kw) * P.Cin) * 2);
    return (k0 + krow0 + i * KSTEP < P.K) ? o : nrec;
  }
};

// EPF: rows the BN-statistics epilogue reads from LDS before storing (2 fits the gather
// loaders' registers without scratch; 4 spills 480-512 B/lane)
template <int BM, int BN, template <int, int, int> class LA, template <int, int, int> class LB, int EPI,
          int EPF = 1>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) conv_glds_kernel(CoreParams P) {
  mfma_gemm_glds<BM, BN, 2, 2, LA, LB, EPI, 1, EPF>(P);
}

// 8 waves (2 x 4, wave tile 64 x BN/4) with a double-buffered LDS-DMA pipeline:
// same 16 waves/CU occupancy as the 4-wave single-stage kernel, but the next K
// tile's DMA overlaps this tile's MFMAs (CLOUD_AMD_GEMM_CORE=glds8).
template <int BM, int BN, template <int, int, int> class LA, template <int, int, int> class LB, int EPI>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) conv_glds8_kernel(CoreParams P) {
  mfma_gemm_glds<BM, BN, 2, 4, LA, LB, EPI, 2>(P);
}

// Tall tiles for the <= 64-channel implicit-GEMM convolutions (ResNet layer-1 3x3 fwd and
// dgrad): 256 x 64 with 4 x 1 waves (64 x 64 wave tiles) -- twice the MFMAs per K-tile
// barrier of the 128 x 64 / 2 x 2 tile and one B-operand fetch per 256 rows.
template <int BM, int BN, int WM, int WN, template <int, int, int> class LA, template <int, int, int> class LB,
          int EPI, int EPF = 1>
__global__ void __launch_bounds__(WM * WN * 64) __attribute__((amdgpu_waves_per_eu(4)))
conv_glds_w_kernel(CoreParams P) {
  mfma_gemm_glds<BM, BN, WM, WN, LA, LB, EPI, 1, EPF>(P);
}

// Forward convolutions with the BN-statistics epilogue read 2 staged rows per epilogue trip
// (fwd3x3 -2..-5 % per call, end-to-end neutral: 14,148 vs 14,137 img/s same box);
// CLOUD_AMD_CONV_EPI_PF=0 restores one row per trip (A/B runs).
bool conv_epi_pf() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CLOUD_AMD_CONV_EPI_PF");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v != 0;
}

// CLOUD_AMD_CONV_TALL=0 keeps 128 x 64 tiles on those convolutions (A/B runs).
bool tall_tiles() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CLOUD_AMD_CONV_TALL");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v != 0;
}

// The space-to-depth stem (K = 3 row tiles, N = 64) on the tall 256 x 64 tiles as well: 0.88 ->
// 0.72 ms per call at b1024 (profiles/r4_s34/); CLOUD_AMD_STEM_TALL=0 keeps 128 x 64 (A/B runs)
bool stem_tall() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CLOUD_AMD_STEM_TALL");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v != 0;
}

// CLOUD_AMD_GEMM_CORE=reg selects the register-staged core (A/B comparisons).
// 0 = register-staged, 1 = glds single stage (4 waves), 2 = glds double-buffered (8 waves)
int core_kind() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CLOUD_AMD_GEMM_CORE");
    v = !e ? 1 : (e[0] == 'r' ? 0 : (strcmp(e, "glds8") == 0 ? 2 : 1));
  }
  return v;
}
bool use_glds() { return core_kind() != 0; }

// CLOUD_AMD_TAPMASK=0 keeps the general gather loaders on every convolution (A/B runs).
bool tapmask_loaders() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CLOUD_AMD_TAPMASK");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v != 0;
}

template <int BM, int BN, template <int, int, int> class LA, template <int, int, int> class LB, int EPI>
__global__ void __launch_bounds__(256) conv_gemm_kernel(CoreParams P) {
  mfma_gemm_body<BM, BN, 2, 2, LA, LB, EPI, 2>(P);
}

template <int BM, int BN, template <int, int, int> class LA, template <int, int, int> class LB,
          template <int, int, int> class GA, template <int, int, int> class GB, int EPI>
int launch(const CoreParams& p0, int splits, hipStream_t s) {
  CoreParams p = p0;
  p.split_xcd = split_xcd_enabled();
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  if (BN == 128 && core_kind() == 2) {
    conv_glds8_kernel<BM, BN, GA, GB, EPI><<<dim3(tiles, 1, splits), 512, 0, s>>>(p);
    CA_LAUNCH_CHECK();
    return 0;
  }
  if constexpr (EPI == EPI_BF16_ST) {
    if (use_glds() && conv_epi_pf()) {
      conv_glds_kernel<BM, BN, GA, GB, EPI, 2><<<dim3(tiles, 1, splits), 256, 0, s>>>(p);
      CA_LAUNCH_CHECK();
      return 0;
    }
  }
  if (use_glds()) {
    conv_glds_kernel<BM, BN, GA, GB, EPI><<<dim3(tiles, 1, splits), 256, 0, s>>>(p);
    CA_LAUNCH_CHECK();
    return 0;
  }
  conv_gemm_kernel<BM, BN, LA, LB, EPI><<<dim3(tiles, 1, splits), 256, 0, s>>>(p);
  CA_LAUNCH_CHECK();
  return 0;
}

// 128 x 64 launch of an N <= 64 convolution, as 256 x 64 / 4 x 1 waves when enabled
template <template <int, int, int> class LA, template <int, int, int> class LB,
          template <int, int, int> class GA, template <int, int, int> class GB, int EPI>
int launch_n64(const CoreParams& p0, hipStream_t s) {
  if (!(tall_tiles() && core_kind() == 1)) return launch<128, 64, LA, LB, GA, GB, EPI>(p0, 1, s);
  CoreParams p = p0;
  p.split_xcd = split_xcd_enabled();
  const int tiles = (p.M + 255) / 256;
  if constexpr (EPI == EPI_BF16_ST) {
    if (conv_epi_pf()) {
      conv_glds_w_kernel<256, 64, 4, 1, GA, GB, EPI, 2><<<dim3(tiles, 1, 1), 256, 0, s>>>(p);
      CA_LAUNCH_CHECK();
      return 0;
    }
  }
  conv_glds_w_kernel<256, 64, 4, 1, GA, GB, EPI><<<dim3(tiles, 1, 1), 256, 0, s>>>(p);
  CA_LAUNCH_CHECK();
  return 0;
}

// 3x3 / s1 / p1 / 64-channel convolutions at width 56 (ResNet-50 stage-1 conv2, forward and
// input gradient) on the LDS-resident patch + filter kernel (csrc/include/ca_conv_halo.h);
// CLOUD_AMD_CONV_HALO=0 keeps them on the implicit-GEMM kernels, =2 runs the halo kernel
// without the software-pipelined fragment reads (A/B runs).
template <int STATS, bool PIPE>
__global__ void __launch_bounds__(HALO_NT) conv3x3_halo_kernel(HaloParams P) {
  conv3x3_halo<STATS, PIPE>(P);
}

int halo_mode() {
  static int en = -1;
  if (en < 0) {
    const char* e = getenv("CLOUD_AMD_CONV_HALO");
    en = !e ? 1 : (e[0] == '0' ? 0 : (e[0] == '2' ? 2 : 1));
  }
  return en;
}

bool halo_shape(int H, int W, int Cin, int Cout, int KH, int KW, int sh, int sw, int ph, int pw) {
  const int en = halo_mode();
  return en && KH == 3 && KW == 3 && sh == 1 && sw == 1 && ph == 1 && pw == 1 && Cin == HALO_C && Cout == HALO_C &&
         W == 56 && H % HALO_TR == 0 && use_glds();
}

// persistent grid: one workgroup per CU (the 148-KB LDS image), at most one per tile
int conv_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    hipDeviceProp_t prop;
    cus = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess &&
           prop.multiProcessorCount > 0) ? prop.multiProcessorCount : 256;
  }
  return cus;
}

int halo_grid(int Nb, int H) {
  const int cus = conv_cus();
  const long tiles = (long)Nb * (H / HALO_TR);
  return (int)(tiles < cus ? tiles : cus);
}

__global__ void __launch_bounds__(HWG_NT) conv3x3_halo_wgrad_kernel(HaloWgParams P) { conv3x3_halo_wgrad(P); }

// weight gradient on the halo kernel: CLOUD_AMD_CONV_HALO_WGRAD=0 keeps the implicit GEMM
bool halo_wgrad_on() {
  static int en = -1;
  if (en < 0) {
    const char* e = getenv("CLOUD_AMD_CONV_HALO_WGRAD");
    en = (e && e[0] == '0') ? 0 : 1;
  }
  return en != 0;
}

int halo_launch(const bf16_t* x, const bf16_t* w, bf16_t* y, int Nb, int H, int W, float* stats, const bf16_t* bnz,
                const uint8_t* bnmask, int dgrad, hipStream_t s) {
  HaloParams hp{};
  hp.x = x; hp.w = w; hp.y = y; hp.stats = stats; hp.bnz = bnz; hp.bnmask = bnmask;
  hp.N = Nb; hp.H = H; hp.W = W; hp.dgrad = dgrad;
  const int g = halo_grid(Nb, H);
  const bool pipe = halo_mode() != 2;
  const int mode = stats ? (dgrad ? 2 : 1) : 0;
  if (pipe) {
    if (mode == 2) conv3x3_halo_kernel<2, true><<<g, HALO_NT, 0, s>>>(hp);
    else if (mode == 1) conv3x3_halo_kernel<1, true><<<g, HALO_NT, 0, s>>>(hp);
    else conv3x3_halo_kernel<0, true><<<g, HALO_NT, 0, s>>>(hp);
  } else {
    if (mode == 2) conv3x3_halo_kernel<2, false><<<g, HALO_NT, 0, s>>>(hp);
    else if (mode == 1) conv3x3_halo_kernel<1, false><<<g, HALO_NT, 0, s>>>(hp);
    else conv3x3_halo_kernel<0, false><<<g, HALO_NT, 0, s>>>(hp);
  }
  CA_LAUNCH_CHECK();
  return 0;
}

// Space-to-depth stem (4x4 / s1 / p0, 16 -> 64 channels, output width 112) on the LDS-resident
// patch + filter kernel (csrc/include/ca_conv_stem.h); CLOUD_AMD_STEM_LDS=0 keeps it on the
// implicit-GEMM row-segment loader (A/B runs).
template <bool STATS>
__global__ void __launch_bounds__(STEM_NT) conv_stem_s2d_kernel(StemParams P) {
  conv_stem_s2d<STATS>(P);
}

bool stem_lds_on() {
  static int en = -1;
  if (en < 0) {
    const char* e = getenv("CLOUD_AMD_STEM_LDS");
    en = (e && e[0] == '0') ? 0 : 1;
  }
  return en != 0;
}

bool stem_shape(int H, int W, int Cin, int Cout, int KH, int KW, int sh, int sw, int ph, int pw) {
  return stem_lds_on() && KH == 4 && KW == 4 && sh == 1 && sw == 1 && ph == 0 && pw == 0 && Cin == STEM_CI &&
         Cout == STEM_C && W == STEM_PW && H > 3 && (H - 3) % STEM_TR == 0;
}

// persistent grid: one workgroup per CU (196 VGPRs per lane: a second 7-wave workgroup does
// not fit the register file), at most one per tile
int stem_grid(int Nb, int H) {
  const long tiles = (long)Nb * ((H - 3) / STEM_TR);
  const long g = conv_cus();
  return (int)(tiles < g ? tiles : g);
}

int stem_launch(const bf16_t* x, const bf16_t* w, bf16_t* y, int Nb, int H, float* stats, hipStream_t s) {
  StemParams sp{};
  sp.x = x; sp.w = w; sp.y = y; sp.stats = stats; sp.N = Nb; sp.OH = H - 3;
  const int g = stem_grid(Nb, H);
  if (stats) conv_stem_s2d_kernel<true><<<g, STEM_NT, 0, s>>>(sp);
  else conv_stem_s2d_kernel<false><<<g, STEM_NT, 0, s>>>(sp);
  CA_LAUNCH_CHECK();
  return 0;
}

CoreParams conv_params(int Nb, int H, int W, int Cin, int Cout, int KH, int KW, int sh, int sw, int ph, int pw) {
  CoreParams p{};
  p.Nb = Nb; p.H = H; p.W = W; p.Cin = Cin; p.Cout = Cout; p.KH = KH; p.KW = KW;
  p.sh = sh; p.sw = sw; p.ph = ph; p.pw = pw;
  p.OH = (H + 2 * ph - KH) / sh + 1;
  p.OW = (W + 2 * pw - KW) / sw + 1;
  p.div_ow = make_fastdiv(p.OW); p.div_oh = make_fastdiv(p.OH);
  p.div_w = make_fastdiv(W); p.div_h = make_fastdiv(H);
  p.div_cin = make_fastdiv(Cin); p.div_cout = make_fastdiv(Cout); p.div_kw = make_fastdiv(KW);
  p.cin_tile = (Cin % BK == 0) ? 1 : 0;
  p.cout_tile = (Cout % BK == 0) ? 1 : 0;
  return p;
}

bool geom_ok(int Cin, int Cout, long pixels) {
  return Cin >= 8 && Cout >= 8 && Cin % 8 == 0 && Cout % 8 == 0 && pixels > 0 && pixels < (1L << 31);
}

}  // namespace

extern "C" int ca_splitk_reduce(const float*, int, long, void*, int, float, hipStream_t);

extern "C" {

// y[Nb,OH,OW,Cout] = conv(x[Nb,H,W,Cin], w[Cout,KH,KW,Cin]); optional BN-stat partials.
int ca_conv_fwd(const bf16_t* x, const bf16_t* w, bf16_t* y, int Nb, int H, int W, int Cin, int Cout, int KH,
                int KW, int sh, int sw, int ph, int pw, float* stats, hipStream_t s) {
  CoreParams p = conv_params(Nb, H, W, Cin, Cout, KH, KW, sh, sw, ph, pw);
  if (!geom_ok(Cin, Cout, (long)Nb * H * W)) return -1;
  if (halo_shape(H, W, Cin, Cout, KH, KW, sh, sw, ph, pw))
    return halo_launch(x, w, y, Nb, H, W, stats, nullptr, nullptr, 0, s);
  if (stem_shape(H, W, Cin, Cout, KH, KW, sh, sw, ph, pw) && use_glds()) return stem_launch(x, w, y, Nb, H, stats, s);
  p.A = x; p.B = w; p.lda = Cin; p.ldb = (long)KH * KW * Cin; p.C = y; p.ldc = Cout;
  p.M = Nb * p.OH * p.OW; p.N = Cout; p.K = KH * KW * Cin; p.k_per_split = p.K;
  p.stats = stats;
  if (sh == 1 && sw == 1 && ph == 0 && pw == 0 && KW * Cin == BK && tapmask_loaders() && use_glds() &&
      (long)Nb * H * W * Cin * 2 < (long)BUF_CAP) {
    // one K tile per kernel row (the space-to-depth stem): row-segment loader
    if (Cout <= 64 && stem_tall())
      return stats ? launch_n64<ConvFwdA, DenseKC, GConvRowA, GDenseKC, EPI_BF16_ST>(p, s)
                   : launch_n64<ConvFwdA, DenseKC, GConvRowA, GDenseKC, EPI_BF16>(p, s);
    if (Cout <= 64)
      return stats ? launch<128, 64, ConvFwdA, DenseKC, GConvRowA, GDenseKC, EPI_BF16_ST>(p, 1, s)
                   : launch<128, 64, ConvFwdA, DenseKC, GConvRowA, GDenseKC, EPI_BF16>(p, 1, s);
    return stats ? launch<128, 128, ConvFwdA, DenseKC, GConvRowA, GDenseKC, EPI_BF16_ST>(p, 1, s)
                 : launch<128, 128, ConvFwdA, DenseKC, GConvRowA, GDenseKC, EPI_BF16>(p, 1, s);
  }
  if (p.cin_tile && KH * KW <= 32 && tapmask_loaders()) {
    if (stats) {
      if (Cout <= 64) return launch_n64<ConvFwdA, DenseKC, GConvFwdAT, GDenseKC, EPI_BF16_ST>(p, s);
      return launch<128, 128, ConvFwdA, DenseKC, GConvFwdAT, GDenseKC, EPI_BF16_ST>(p, 1, s);
    }
    if (Cout <= 64) return launch_n64<ConvFwdA, DenseKC, GConvFwdAT, GDenseKC, EPI_BF16>(p, s);
    return launch<128, 128, ConvFwdA, DenseKC, GConvFwdAT, GDenseKC, EPI_BF16>(p, 1, s);
  }
  if (stats) {
    if (Cout <= 64) return launch<128, 64, ConvFwdA, DenseKC, GConvFwdA, GDenseKC, EPI_BF16_ST>(p, 1, s);
    return launch<128, 128, ConvFwdA, DenseKC, GConvFwdA, GDenseKC, EPI_BF16_ST>(p, 1, s);
  }
  if (Cout <= 64) return launch<128, 64, ConvFwdA, DenseKC, GConvFwdA, GDenseKC, EPI_BF16>(p, 1, s);
  return launch<128, 128, ConvFwdA, DenseKC, GConvFwdA, GDenseKC, EPI_BF16>(p, 1, s);
}

// Keras Conv2D forward: y = act(conv(x, w) + bias) with bias [Cout] fp32 (or null) and
// act one of the core's ACT_* codes, applied in the bf16 epilogue (no separate passes).
int ca_conv_fwd_ex(const bf16_t* x, const bf16_t* w, bf16_t* y, int Nb, int H, int W, int Cin, int Cout, int KH,
                   int KW, int sh, int sw, int ph, int pw, const float* bias, int act, hipStream_t s) {
  CoreParams p = conv_params(Nb, H, W, Cin, Cout, KH, KW, sh, sw, ph, pw);
  if (!geom_ok(Cin, Cout, (long)Nb * H * W)) return -1;
  p.A = x; p.B = w; p.lda = Cin; p.ldb = (long)KH * KW * Cin; p.C = y; p.ldc = Cout;
  p.M = Nb * p.OH * p.OW; p.N = Cout; p.K = KH * KW * Cin; p.k_per_split = p.K;
  p.bias = bias;
  p.act = act;
  if (Cout <= 64) return launch<128, 64, ConvFwdA, DenseKC, GConvFwdA, GDenseKC, EPI_BF16>(p, 1, s);
  return launch<128, 128, ConvFwdA, DenseKC, GConvFwdA, GDenseKC, EPI_BF16>(p, 1, s);
}

// Rows of the BN-backward statistics partials ca_conv_dgrad_bnstats writes: one per
// 128-row GEMM tile, summed over the output-parity classes of a strided dgrad.
long ca_conv_dgrad_stat_tiles(int Nb, int H, int W, int sh, int sw);

// Rows of the BN-forward statistics partials ca_conv_fwd(stats != null) writes: one per
// 128 output pixels on the implicit-GEMM kernels, one per workgroup on the halo and stem kernels.
long ca_conv_stat_rows(int Nb, int H, int W, int Cin, int Cout, int KH, int KW, int sh, int sw, int ph, int pw) {
  if (halo_shape(H, W, Cin, Cout, KH, KW, sh, sw, ph, pw)) return halo_grid(Nb, H);
  if (stem_shape(H, W, Cin, Cout, KH, KW, sh, sw, ph, pw) && use_glds()) return stem_grid(Nb, H);
  const long oh = (H + 2 * ph - KH) / sh + 1, ow = (W + 2 * pw - KW) / sw + 1;
  return ((long)Nb * oh * ow + 127) / 128;
}

// Rows of ca_conv_dgrad_bnstats' partials for the full geometry (the halo kernel writes one
// per workgroup; beta must be 0 for it to run).
long ca_conv_dgrad_stat_rows(int Nb, int H, int W, int Cin, int Cout, int KH, int KW, int sh, int sw, int ph, int pw,
                             float beta) {
  if (beta == 0.f && halo_shape(H, W, Cin, Cout, KH, KW, sh, sw, ph, pw)) return halo_grid(Nb, H);
  return ca_conv_dgrad_stat_tiles(Nb, H, W, sh, sw);
}

long ca_conv_dgrad_stat_tiles(int Nb, int H, int W, int sh, int sw) {
  if ((sh == 1 && sw == 1) || !use_glds()) return ((long)Nb * H * W + 127) / 128;
  long t = 0;
  for (int py = 0; py < sh; ++py)
    for (int px = 0; px < sw; ++px) {
      const long hq = (H - py + sh - 1) / sh, wq = (W - px + sw - 1) / sw;
      if (hq > 0 && wq > 0) t += ((long)Nb * hq * wq + 127) / 128;
    }
  return t;
}

}  // extern "C"

template <int EPI>
static int launch_dgrad(const CoreParams& p, int Cin, hipStream_t s) {
  if (p.cout_tile && p.sh == 1 && p.sw == 1 && p.KH * p.KW <= 32 && tapmask_loaders()) {
    if (Cin <= 64) return launch_n64<ConvDgradA, ConvDgradB, GConvDgradAT, GConvDgradBT, EPI>(p, s);
    return launch<128, 128, ConvDgradA, ConvDgradB, GConvDgradAT, GConvDgradBT, EPI>(p, 1, s);
  }
  if (Cin <= 64) return launch<128, 64, ConvDgradA, ConvDgradB, GConvDgradA, GConvDgradB, EPI>(p, 1, s);
  return launch<128, 128, ConvDgradA, ConvDgradB, GConvDgradA, GConvDgradB, EPI>(p, 1, s);
}

// one output-parity class of a strided dgrad (row map on)
template <int EPI>
static int launch_dgrad_s(const CoreParams& q, int Cin, hipStream_t s) {
  if (q.cout_tile && q.dg_nh * q.dg_nw <= 32 && tapmask_loaders()) {
    if (Cin <= 64) return launch<128, 64, ConvDgradA, ConvDgradB, GConvDgradSAT, GConvDgradSBT, EPI>(q, 1, s);
    return launch<128, 128, ConvDgradA, ConvDgradB, GConvDgradSAT, GConvDgradSBT, EPI>(q, 1, s);
  }
  if (Cin <= 64) return launch<128, 64, ConvDgradA, ConvDgradB, GConvDgradSA, GConvDgradSB, EPI>(q, 1, s);
  return launch<128, 128, ConvDgradA, ConvDgradB, GConvDgradSA, GConvDgradSB, EPI>(q, 1, s);
}

static int conv_dgrad_impl(const bf16_t* dy, const bf16_t* w, bf16_t* dx, int Nb, int H, int W, int Cin, int Cout,
                           int KH, int KW, int sh, int sw, int ph, int pw, float beta, const bf16_t* bnz,
                           const uint8_t* bnmask, float* stats, hipStream_t s, int skip_empty = 0) {
  CoreParams p = conv_params(Nb, H, W, Cin, Cout, KH, KW, sh, sw, ph, pw);
  if (!geom_ok(Cin, Cout, (long)Nb * H * W)) return -1;
  if (beta == 0.f && halo_shape(H, W, Cin, Cout, KH, KW, sh, sw, ph, pw))
    return halo_launch(dy, w, dx, Nb, H, W, bnz ? stats : nullptr, bnz, bnmask, 1, s);
  p.A = dy; p.B = w; p.C = dx; p.ldc = Cin;
  p.M = Nb * H * W; p.N = Cin; p.K = KH * KW * Cout; p.k_per_split = p.K;
  p.beta = beta;
  p.bnz = bnz;
  p.bnmask = bnmask;
  p.stats = bnz ? stats : nullptr;
  if ((sh > 1 || sw > 1) && use_glds()) {
    long stat_row = 0;
    // one GEMM per output-parity class; classes without taps get zeros (or beta*dx)
    for (int py = 0; py < sh; ++py)
      for (int px = 0; px < sw; ++px) {
        CoreParams q = p;
        q.rowmap = 1;
        q.dg_py = py;
        q.dg_px = px;
        q.dg_kh0 = (py + ph) % sh;
        q.dg_kw0 = (px + pw) % sw;
        q.dg_nh = q.dg_kh0 < KH ? (KH - q.dg_kh0 + sh - 1) / sh : 0;
        q.dg_nw = q.dg_kw0 < KW ? (KW - q.dg_kw0 + sw - 1) / sw : 0;
        q.dg_dy0 = (py + ph - q.dg_kh0) / sh;
        q.dg_dx0 = (px + pw - q.dg_kw0) / sw;
        q.Hq = (H - py + sh - 1) / sh;
        q.Wq = (W - px + sw - 1) / sw;
        if (q.Hq <= 0 || q.Wq <= 0) continue;
        // skip_empty: a class no tap reaches keeps its pixels unwritten (the caller's next
        // GEMM into dx reads them as zeros: CoreParams::bpar_s)
        if (skip_empty && q.dg_nh * q.dg_nw == 0) continue;
        q.div_hq = make_fastdiv(q.Hq);
        q.div_wq = make_fastdiv(q.Wq);
        q.div_nw = make_fastdiv(q.dg_nw > 0 ? q.dg_nw : 1);
        q.M = Nb * q.Hq * q.Wq;
        q.K = q.dg_nh * q.dg_nw * Cout;
        q.k_per_split = q.K;
        if (bnz) {
          q.stats = stats + stat_row * 2 * Cin;  // this class's tiles follow the previous classes'
          stat_row += (q.M + 127) / 128;
        }
        int rc = bnz ? launch_dgrad_s<EPI_BF16_BN>(q, Cin, s) : launch_dgrad_s<EPI_BF16>(q, Cin, s);
        if (rc) return rc;
      }
    return 0;
  }
  return bnz ? launch_dgrad<EPI_BF16_BN>(p, Cin, s) : launch_dgrad<EPI_BF16>(p, Cin, s);
}

extern "C" {

// dx[Nb,H,W,Cin] = dgrad(dy[Nb,OH,OW,Cout], w) (+ beta * dx).
// skip_empty (strided, beta 0 only): output-parity classes without taps are left unwritten
// instead of zero-filled.
int ca_conv_dgrad(const bf16_t* dy, const bf16_t* w, bf16_t* dx, int Nb, int H, int W, int Cin, int Cout, int KH,
                  int KW, int sh, int sw, int ph, int pw, float beta, hipStream_t s, int skip_empty) {
  if (skip_empty && (beta != 0.f || (sh == 1 && sw == 1))) return -1;
  // (the non-LDS-DMA loaders run one implicit GEMM over every pixel: it writes the empty
  // classes' zeros anyway, which a sparse-beta reader may equally skip)
  return conv_dgrad_impl(dy, w, dx, Nb, H, W, Cin, Cout, KH, KW, sh, sw, ph, pw, beta, nullptr, nullptr, nullptr, s,
                         skip_empty);
}

// Same, plus the BN-backward statistics epilogue (see ca_gemm_bf16_bnstats): `stats`
// has ca_conv_dgrad_stat_tiles(...) rows of [2][Cin]; z / mask are indexed like dx.
int ca_conv_dgrad_bnstats(const bf16_t* dy, const bf16_t* w, bf16_t* dx, int Nb, int H, int W, int Cin, int Cout,
                          int KH, int KW, int sh, int sw, int ph, int pw, float beta, const bf16_t* bnz,
                          const uint8_t* bnmask, float* stats, hipStream_t s) {
  if (!bnz || !stats) return -1;
  return conv_dgrad_impl(dy, w, dx, Nb, H, W, Cin, Cout, KH, KW, sh, sw, ph, pw, beta, bnz, bnmask, stats, s);
}

// dw[Cout, KH*KW*Cin] (+)= wgrad(dy, x) via split-K fp32 slabs in ws[splits][Cout][KH*KW*Cin].
int ca_conv_wgrad(const bf16_t* dy, const bf16_t* x, void* dw, int dw_bf16, float beta, int Nb, int H, int W,
                  int Cin, int Cout, int KH, int KW, int sh, int sw, int ph, int pw, int splits, float* ws,
                  hipStream_t s) {
  if (halo_shape(H, W, Cin, Cout, KH, KW, sh, sw, ph, pw) && halo_wgrad_on() && splits == halo_grid(Nb, H)) {
    // one fp32 [64][576] partial per persistent workgroup (ca_conv_wgrad_splits sized ws)
    HaloWgParams hp{x, dy, ws, Nb, H, W};
    conv3x3_halo_wgrad_kernel<<<splits, HWG_NT, 0, s>>>(hp);
    CA_LAUNCH_CHECK();
    return ca_splitk_reduce(ws, splits, (long)Cout * KH * KW * Cin, dw, dw_bf16, beta, s);
  }
  CoreParams p = conv_params(Nb, H, W, Cin, Cout, KH, KW, sh, sw, ph, pw);
  if (!geom_ok(Cin, Cout, (long)Nb * H * W)) return -1;
  p.A = dy; p.lda = Cout; p.B = x;
  p.M = Cout; p.N = KH * KW * Cin; p.K = Nb * p.OH * p.OW;
  int kps = (p.K / splits + BK - 1) / BK * BK;
  if (kps < BK) kps = BK;
  splits = (p.K + kps - 1) / kps;
  p.k_per_split = kps;
  p.C = ws; p.ldc = p.N; p.split_stride = (long)p.M * p.N;
  int rc;
  if (tapmask_loaders() && (long)p.OH * p.OW >= 2 * BK) {  // incremental pixel walk (GConvWgradBI)
    if (Cout <= 64)
      rc = (p.N <= 64) ? launch<64, 64, DenseNC, ConvWgradB, GDenseNC, GConvWgradBI, EPI_F32_PARTIAL>(p, splits, s)
                       : launch<64, 128, DenseNC, ConvWgradB, GDenseNC, GConvWgradBI, EPI_F32_PARTIAL>(p, splits, s);
    else
      rc = (p.N <= 64) ? launch<128, 64, DenseNC, ConvWgradB, GDenseNC, GConvWgradBI, EPI_F32_PARTIAL>(p, splits, s)
                       : launch<128, 128, DenseNC, ConvWgradB, GDenseNC, GConvWgradBI, EPI_F32_PARTIAL>(p, splits, s);
    if (rc) return rc;
    return ca_splitk_reduce(ws, splits, (long)p.M * p.N, dw, dw_bf16, beta, s);
  }
  if (tapmask_loaders()) {
    if (Cout <= 64)
      rc = (p.N <= 64) ? launch<64, 64, DenseNC, ConvWgradB, GDenseNC, GConvWgradBT, EPI_F32_PARTIAL>(p, splits, s)
                       : launch<64, 128, DenseNC, ConvWgradB, GDenseNC, GConvWgradBT, EPI_F32_PARTIAL>(p, splits, s);
    else
      rc = (p.N <= 64) ? launch<128, 64, DenseNC, ConvWgradB, GDenseNC, GConvWgradBT, EPI_F32_PARTIAL>(p, splits, s)
                       : launch<128, 128, DenseNC, ConvWgradB, GDenseNC, GConvWgradBT, EPI_F32_PARTIAL>(p, splits, s);
    if (rc) return rc;
    return ca_splitk_reduce(ws, splits, (long)p.M * p.N, dw, dw_bf16, beta, s);
  }
  if (Cout <= 64)  // 64 output channels: 64-row tiles (no MFMA rows past Cout)
    rc = (p.N <= 64) ? launch<64, 64, DenseNC, ConvWgradB, GDenseNC, GConvWgradB, EPI_F32_PARTIAL>(p, splits, s)
                     : launch<64, 128, DenseNC, ConvWgradB, GDenseNC, GConvWgradB, EPI_F32_PARTIAL>(p, splits, s);
  else
    rc = (p.N <= 64) ? launch<128, 64, DenseNC, ConvWgradB, GDenseNC, GConvWgradB, EPI_F32_PARTIAL>(p, splits, s)
                     : launch<128, 128, DenseNC, ConvWgradB, GDenseNC, GConvWgradB, EPI_F32_PARTIAL>(p, splits, s);
  if (rc) return rc;
  return ca_splitk_reduce(ws, splits, (long)p.M * p.N, dw, dw_bf16, beta, s);
}

// Split count (fp32 partial slabs) ca_conv_wgrad will use for this shape: the halo kernel's
// persistent grid where it applies, else `fallback` (the caller's split-K choice).
int ca_conv_wgrad_splits(int Nb, int H, int W, int Cin, int Cout, int KH, int KW, int sh, int sw, int ph, int pw,
                         int fallback) {
  if (halo_shape(H, W, Cin, Cout, KH, KW, sh, sw, ph, pw) && halo_wgrad_on()) return halo_grid(Nb, H);
  return fallback;
}

int ca_conv_out_hw(int H, int KH, int sh, int ph) { return (H + 2 * ph - KH) / sh + 1; }

}  // extern "C"
