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

// A of forward: rows = output pixels, k = (tap, ci).  KC.
template <int R>
struct ConvFwdA {
  static constexpr bool KC = true;
  const CoreParams& P;
  __device__ ConvFwdA(const CoreParams& p, bool) : P(p) {}
  __device__ __forceinline__ s8v load(int r0, int k0, int row, int col) const {
    const int m = r0 + row, k = k0 + col;
    if (m >= P.M || k >= P.K) return zero8();
    const Pix o = decode((uint32_t)m, P.div_ow, P.div_oh);
    const uint32_t tap = fdiv((uint32_t)k, P.div_cin);
    const int ci = k - (int)tap * P.Cin;
    const uint32_t kh = fdiv(tap, P.div_kw);
    const int kw = (int)tap - (int)kh * P.KW;
    const int ih = o.y * P.sh - P.ph + (int)kh, iw = o.x * P.sw - P.pw + kw;
    if ((unsigned)ih >= (unsigned)P.H || (unsigned)iw >= (unsigned)P.W) return zero8();
    return ld16(P.A + (((long)o.n * P.H + ih) * P.W + iw) * P.Cin + ci);
  }
};

// A of dgrad: rows = input pixels, k = (tap, co) over dY.  KC.
template <int R>
struct ConvDgradA {
  static constexpr bool KC = true;
  const CoreParams& P;
  __device__ ConvDgradA(const CoreParams& p, bool) : P(p) {}
  __device__ __forceinline__ s8v load(int r0, int k0, int row, int col) const {
    const int m = r0 + row, k = k0 + col;
    if (m >= P.M || k >= P.K) return zero8();
    const Pix i = decode((uint32_t)m, P.div_w, P.div_h);
    const uint32_t tap = fdiv((uint32_t)k, P.div_cout);
    const int co = k - (int)tap * P.Cout;
    const uint32_t kh = fdiv(tap, P.div_kw);
    const int kw = (int)tap - (int)kh * P.KW;
    int oy = i.y + P.ph - (int)kh, ox = i.x + P.pw - kw;
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
    return ld16(P.A + (((long)i.n * P.OH + oy) * P.OW + ox) * P.Cout + co);
  }
};

// B of dgrad: B[k=(tap,co)][ci] = W[co][tap][ci]  (ci contiguous -> NC).
template <int R>
struct ConvDgradB {
  static constexpr bool KC = false;
  const CoreParams& P;
  __device__ ConvDgradB(const CoreParams& p, bool) : P(p) {}
  __device__ __forceinline__ s8v load(int r0, int k0, int row, int col) const {
    const int k = k0 + row, ci = r0 + col;
    if (k >= P.K || ci >= P.N) return zero8();
    const uint32_t tap = fdiv((uint32_t)k, P.div_cout);
    const int co = k - (int)tap * P.Cout;
    return ld16(P.B + ((long)co * (P.KH * P.KW) + tap) * P.Cin + ci);
  }
};

// B of wgrad: B[k=(n,oh,ow)][j=(tap,ci)] = X[n, oh*s-p+kh, ow*s-p+kw, ci]  (NC).
template <int R>
struct ConvWgradB {
  static constexpr bool KC = false;
  const CoreParams& P;
  __device__ ConvWgradB(const CoreParams& p, bool) : P(p) {}
  __device__ __forceinline__ s8v load(int r0, int k0, int row, int col) const {
    const int k = k0 + row, j = r0 + col;
    if (k >= P.K || j >= P.N) return zero8();
    const Pix o = decode((uint32_t)k, P.div_ow, P.div_oh);
    const uint32_t tap = fdiv((uint32_t)j, P.div_cin);
    const int ci = j - (int)tap * P.Cin;
    const uint32_t kh = fdiv(tap, P.div_kw);
    const int kw = (int)tap - (int)kh * P.KW;
    const int ih = o.y * P.sh - P.ph + (int)kh, iw = o.x * P.sw - P.pw + kw;
    if ((unsigned)ih >= (unsigned)P.H || (unsigned)iw >= (unsigned)P.W) return zero8();
    return ld16(P.B + (((long)o.n * P.H + ih) * P.W + iw) * P.Cin + ci);
  }
};

template <int BM, int BN, class LA, class LB, int EPI>
__global__ void __launch_bounds__(256) conv_gemm_kernel(CoreParams P) {
  mfma_gemm_body<BM, BN, 2, 2, LA, LB, EPI>(P);
}

template <int BM, int BN, class LA, class LB, int EPI>
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
  if (Cout <= 64) return launch<128, 64, ConvFwdA<128>, DenseKC<64>, EPI_BF16>(p, 1, s);
  return launch<128, 128, ConvFwdA<128>, DenseKC<128>, EPI_BF16>(p, 1, s);
}

// dx[Nb,H,W,Cin] = dgrad(dy[Nb,OH,OW,Cout], w) (+ beta * dx).
int ca_conv_dgrad(const bf16_t* dy, const bf16_t* w, bf16_t* dx, int Nb, int H, int W, int Cin, int Cout, int KH,
                  int KW, int sh, int sw, int ph, int pw, float beta, hipStream_t s) {
  CoreParams p = conv_params(Nb, H, W, Cin, Cout, KH, KW, sh, sw, ph, pw);
  if (!geom_ok(Cin, Cout, (long)Nb * H * W)) return -1;
  p.A = dy; p.B = w; p.C = dx; p.ldc = Cin;
  p.M = Nb * H * W; p.N = Cin; p.K = KH * KW * Cout; p.k_per_split = p.K;
  p.beta = beta;
  if (Cin <= 64) return launch<128, 64, ConvDgradA<128>, ConvDgradB<64>, EPI_BF16>(p, 1, s);
  return launch<128, 128, ConvDgradA<128>, ConvDgradB<128>, EPI_BF16>(p, 1, s);
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
  int rc = (p.N <= 64) ? launch<128, 64, DenseNC<128>, ConvWgradB<64>, EPI_F32_PARTIAL>(p, splits, s)
                       : launch<128, 128, DenseNC<128>, ConvWgradB<128>, EPI_F32_PARTIAL>(p, splits, s);
  if (rc) return rc;
  return ca_splitk_reduce(ws, splits, (long)p.M * p.N, dw, dw_bf16, beta, s);
}

int ca_conv_out_hw(int H, int KH, int sh, int ph) { return (H + 2 * ph - KH) / sh + 1; }

}  // extern "C"
