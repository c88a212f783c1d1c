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

template <int BM, int BN, template <int, int, int> class LA, template <int, int, int> class LB, int EPI>
__global__ void __launch_bounds__(256) conv_gemm_kernel(CoreParams P) {
  mfma_gemm_body<BM, BN, 2, 2, LA, LB, EPI, 2>(P);
}

template <int BM, int BN, template <int, int, int> class LA, template <int, int, int> class LB, int EPI>
int launch(const CoreParams& p, int splits, hipStream_t s) {
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  conv_gemm_kernel<BM, BN, LA, LB, EPI><<<dim3(tiles, 1, splits), 256, 0, s>>>(p);
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
  return Cin % 8 == 0 && Cout % 8 == 0 && pixels < (1L << 31);
}

}  // namespace

extern "C" int ca_splitk_reduce(const float*, int, long, void*, int, float, hipStream_t);

extern "C" {

// y[Nb,OH,OW,Cout] = conv(x[Nb,H,W,Cin], w[Cout,KH,KW,Cin]); optional BN-stat partials.
int ca_conv_fwd(const bf16_t* x, const bf16_t* w, bf16_t* y, int Nb, int H, int W, int Cin, int Cout, int KH,
                int KW, int sh, int sw, int ph, int pw, float* stats, hipStream_t s) {
  CoreParams p = conv_params(Nb, H, W, Cin, Cout, KH, KW, sh, sw, ph, pw);
  if (!geom_ok(Cin, Cout, (long)Nb * H * W)) return -1;
  p.A = x; p.B = w; p.lda = Cin; p.ldb = (long)KH * KW * Cin; p.C = y; p.ldc = Cout;
  p.M = Nb * p.OH * p.OW; p.N = Cout; p.K = KH * KW * Cin; p.k_per_split = p.K;
  p.stats = stats;
  if (Cout <= 64) return launch<128, 64, ConvFwdA, DenseKC, EPI_BF16>(p, 1, s);
  return launch<128, 128, ConvFwdA, DenseKC, EPI_BF16>(p, 1, s);
}

// dx[Nb,H,W,Cin] = dgrad(dy[Nb,OH,OW,Cout], w) (+ beta * dx).
int ca_conv_dgrad(const bf16_t* dy, const bf16_t* w, bf16_t* dx, int Nb, int H, int W, int Cin, int Cout, int KH,
                  int KW, int sh, int sw, int ph, int pw, float beta, hipStream_t s) {
  CoreParams p = conv_params(Nb, H, W, Cin, Cout, KH, KW, sh, sw, ph, pw);
  if (!geom_ok(Cin, Cout, (long)Nb * H * W)) return -1;
  p.A = dy; p.B = w; p.C = dx; p.ldc = Cin;
  p.M = Nb * H * W; p.N = Cin; p.K = KH * KW * Cout; p.k_per_split = p.K;
  p.beta = beta;
  if (Cin <= 64) return launch<128, 64, ConvDgradA, ConvDgradB, EPI_BF16>(p, 1, s);
  return launch<128, 128, ConvDgradA, ConvDgradB, EPI_BF16>(p, 1, s);
}

// dw[Cout, KH*KW*Cin] (+)= wgrad(dy, x) via split-K fp32 slabs in ws[splits][Cout][KH*KW*Cin].
int ca_conv_wgrad(const bf16_t* dy, const bf16_t* x, void* dw, int dw_bf16, float beta, int Nb, int H, int W,
                  int Cin, int Cout, int KH, int KW, int sh, int sw, int ph, int pw, int splits, float* ws,
                  hipStream_t s) {
  CoreParams p = conv_params(Nb, H, W, Cin, Cout, KH, KW, sh, sw, ph, pw);
  if (!geom_ok(Cin, Cout, (long)Nb * H * W)) return -1;
  p.A = dy; p.lda = Cout; p.B = x;
  p.M = Cout; p.N = KH * KW * Cin; p.K = Nb * p.OH * p.OW;
  int kps = (p.K / splits + BK - 1) / BK * BK;
  if (kps < BK) kps = BK;
  splits = (p.K + kps - 1) / kps;
  p.k_per_split = kps;
  p.C = ws; p.ldc = p.N; p.split_stride = (long)p.M * p.N;
  int rc = (p.N <= 64) ? launch<128, 64, DenseNC, ConvWgradB, EPI_F32_PARTIAL>(p, splits, s)
                       : launch<128, 128, DenseNC, ConvWgradB, EPI_F32_PARTIAL>(p, splits, s);
  if (rc) return rc;
  return ca_splitk_reduce(ws, splits, (long)p.M * p.N, dw, dw_bf16, beta, s);
}

int ca_conv_out_hw(int H, int KH, int sh, int ph) { return (H + 2 * ph - KH) / sh + 1; }

}  // extern "C"
