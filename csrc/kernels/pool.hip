// NHWC bf16 pooling (K7 in SURVEY.md section 2.7): MaxPool2D forward with a
// 1-byte window-argmax side output, gather-form backward (no atomics: every
// input pixel pulls from the <= ceil(k/s)^2 windows that cover it), and
// global average pooling forward/backward.  All accesses are 8-channel
// (16-byte) vectors; C must be a multiple of 8.
#include "ca_common.h"

namespace {

__global__ void __launch_bounds__(256) maxpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                         uint8_t* __restrict__ idx, int N, int H, int W, int C,
                                                         int OH, int OW, int k, int s, int p) {
  const int CT = C / 8;
  const long total = (long)N * OH * OW * CT;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int vc = (int)(t % CT);
    long r = t / CT;
    const int ow = (int)(r % OW); r /= OW;
    const int oh = (int)(r % OH);
    const int n = (int)(r / OH);
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
    for (int kh = 0; kh < k; ++kh) {
      const int h = oh * s - p + kh;
      if (h < 0 || h >= H) continue;
      for (int kw = 0; kw < k; ++kw) {
        const int w = ow * s - p + kw;
        if (w < 0 || w >= W) continue;
        us8 v = *reinterpret_cast<const us8*>(x + (((long)n * H + h) * W + w) * C + vc * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float f = bf2f(v[j]);
          if (f > best[j]) { best[j] = f; bi[j] = (uint8_t)(kh * k + kw); }
        }
      }
    }
    us8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(best[j]);
    const long oo = (((long)n * OH + oh) * OW + ow) * C + vc * 8;
    *reinterpret_cast<us8*>(y + oo) = o;
    if (idx) {  // the 8 argmax bytes as one 8-B store
      uint64_t packed = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) packed |= (uint64_t)bi[j] << (8 * j);
      *reinterpret_cast<uint64_t*>(idx + oo) = packed;
    }
  }
}

__global__ void __launch_bounds__(256) maxpool_bwd_kernel(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                         bf16_t* __restrict__ dx, int N, int H, int W, int C,
                                                         int OH, int OW, int k, int s, int p) {
  const int CT = C / 8;
  const long total = (long)N * H * W * CT;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int vc = (int)(t % CT);
    long r = t / CT;
    const int w = (int)(r % W); r /= W;
    const int h = (int)(r % H);
    const int n = (int)(r / H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // windows oh with oh*s - p <= h <= oh*s - p + k - 1
    int oh0 = (h + p - k + 1 + s - 1) / s; if (h + p - k + 1 < 0) oh0 = 0;
    int oh1 = (h + p) / s; if (oh1 >= OH) oh1 = OH - 1;
    int ow0 = (w + p - k + 1 + s - 1) / s; if (w + p - k + 1 < 0) ow0 = 0;
    int ow1 = (w + p) / s; if (ow1 >= OW) ow1 = OW - 1;
    for (int oh = oh0; oh <= oh1; ++oh) {
      const int kh = h - (oh * s - p);
      for (int ow = ow0; ow <= ow1; ++ow) {
        const int kw = w - (ow * s - p);
        const uint8_t want = (uint8_t)(kh * k + kw);
        const long oo = (((long)n * OH + oh) * OW + ow) * C + vc * 8;
        us8 g = *reinterpret_cast<const us8*>(dy + oo);
        // 8 argmax bytes as two dwords
        const uint32_t* ip = reinterpret_cast<const uint32_t*>(idx + oo);
        uint32_t i0 = ip[0], i1 = ip[1];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          uint8_t b = (uint8_t)(((j < 4) ? (i0 >> (8 * j)) : (i1 >> (8 * (j - 4)))) & 0xff);
          if (b == want) acc[j] += bf2f(g[j]);
        }
      }
    }
    us8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
    *reinterpret_cast<us8*>(dx + (((long)n * H + h) * W + w) * C + vc * 8) = o;
  }
}

// x [N, HW, C] -> y [N, C] (mean over HW); one thread per (n, 8-channel vector).
template <typename TO>
__global__ void __launch_bounds__(256) gap_fwd_kernel(const bf16_t* __restrict__ x, TO* __restrict__ y, int N, int HW, int C) {
  const int CT = C / 8;
  const long total = (long)N * CT;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int vc = (int)(t % CT);
    const int n = (int)(t / CT);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const bf16_t* base = x + (long)n * HW * C + vc * 8;
    for (int i = 0; i < HW; ++i) {
      us8 v = *reinterpret_cast<const us8*>(base + (long)i * C);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[j]);
    }
    const float inv = 1.f / (float)HW;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (sizeof(TO) == 2) y[(long)n * C + vc * 8 + j] = f2bf(acc[j] * inv);
      else y[(long)n * C + vc * 8 + j] = acc[j] * inv;
    }
  }
}

template <typename TI>
__global__ void __launch_bounds__(256) gap_bwd_kernel(const TI* __restrict__ dy, bf16_t* __restrict__ dx, int N, int HW, int C) {
  const int CT = C / 8;
  const long total = (long)N * HW * CT;
  const float inv = 1.f / (float)HW;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int vc = (int)(t % CT);
    const long r = t / CT;
    const int n = (int)(r / HW);
    us8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float g;
      if constexpr (sizeof(TI) == 2) g = bf2f(dy[(long)n * C + vc * 8 + j]);
      else g = dy[(long)n * C + vc * 8 + j];
      o[j] = f2bf(g * inv);
    }
    *reinterpret_cast<us8*>(dx + r * C + vc * 8) = o;
  }
}

// Global max pool (Keras GlobalMaxPooling2D = reduce_max over H, W): y[n][c] = max_hw x, and
// cnt[n][c] = how many positions attain it, so the backward splits the gradient evenly
// over ties exactly as reduce_max's gradient (TF) / amax's (torch) does -- an all-zero
// post-ReLU channel is an HW-way tie.  One thread per (n, 8-channel vector).
__global__ void __launch_bounds__(256) gmp_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                      float* __restrict__ cnt, int N, int HW, int C) {
  const int CT = C / 8;
  const long total = (long)N * CT;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int vc = (int)(t % CT);
    const int n = (int)(t / CT);
    float m[8], k[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      m[j] = -INFINITY;
      k[j] = 0.f;
    }
    const bf16_t* base = x + (long)n * HW * C + vc * 8;
    for (int i = 0; i < HW; ++i) {
      const us8 v = *reinterpret_cast<const us8*>(base + (long)i * C);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float f = bf2f(v[j]);
        if (f > m[j]) {
          m[j] = f;
          k[j] = 1.f;
        } else if (f == m[j]) {
          k[j] += 1.f;
        }
      }
    }
    us8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] = f2bf(m[j]);
      cnt[(long)n * C + vc * 8 + j] = k[j];
    }
    *reinterpret_cast<us8*>(y + (long)n * C + vc * 8) = o;
  }
}

// dx = (x == y) * dy / cnt, written for every input element (no separate zero fill)
template <typename TI>
__global__ void __launch_bounds__(256) gmp_bwd_kernel(const TI* __restrict__ dy, const bf16_t* __restrict__ x,
                                                      const bf16_t* __restrict__ y, const float* __restrict__ cnt,
                                                      bf16_t* __restrict__ dx, int N, int HW, int C) {
  const int CT = C / 8;
  const long total = (long)N * HW * CT;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int vc = (int)(t % CT);
    const long r = t / CT;
    const int n = (int)(r / HW);
    const us8 xv = *reinterpret_cast<const us8*>(x + r * C + vc * 8);
    const us8 yv = *reinterpret_cast<const us8*>(y + (long)n * C + vc * 8);
    us8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const long i = (long)n * C + vc * 8 + j;
      float g;
      if constexpr (sizeof(TI) == 2) g = bf2f(dy[i]);
      else g = dy[i];
      o[j] = xv[j] == yv[j] ? f2bf(g / cnt[i]) : (bf16_t)0;
    }
    *reinterpret_cast<us8*>(dx + r * C + vc * 8) = o;
  }
}

}  // namespace

// Space-to-depth of the network input for the 7x7/2 stem (pad 3):
//   y[n, i, j, (by*2 + bx)*4 + c] = x[n, 2i + by - pad, 2j + bx - pad, c]   (c < C <= 4; else / outside: 0)
// turns the stride-2 7x7 conv into a stride-1 4x4 conv over 16 channels (K = 256
// instead of 7*7*8 = 392 with the 8-channel padded input).  One thread per output
// pixel: 16 bf16 = two 16-B stores.
__global__ void __launch_bounds__(256) stem_s2d_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int N,
                                                       int H, int W, int C, int Hs, int Ws, int pad) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)N * Hs * Ws;
  if (idx >= total) return;
  const int j = (int)(idx % Ws);
  const long t = idx / Ws;
  const int i = (int)(t % Hs);
  const int n = (int)(t / Hs);
  us8 out[2];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int by = q >> 1, bx = q & 1;
    const int u = 2 * i + by - pad, v = 2 * j + bx - pad;
    const bool ok = (unsigned)u < (unsigned)H && (unsigned)v < (unsigned)W;
    const bf16_t* src = x + (((long)n * H + (ok ? u : 0)) * W + (ok ? v : 0)) * C;
#pragma unroll
    for (int c = 0; c < 4; ++c) out[q >> 1][(q & 1) * 4 + c] = (ok && c < C) ? src[c] : (bf16_t)0;
  }
  us8* dst = reinterpret_cast<us8*>(y + idx * 16);
  dst[0] = out[0];
  dst[1] = out[1];
}

// Backward of the 3x3 / stride 2 / pad 1 max-pool (the ResNet stem): one thread per
// 2x2 block of input pixels (8 channels).  Input rows 2i, 2i+1 are covered only by
// windows oh = i, i+1 (row 2i by oh = i alone), likewise for columns, so the thread
// reads the <= 4 windows' gradients and argmax bytes once and writes 4 outputs --
// the generic gather re-reads each window for every input pixel it covers.
__global__ void __launch_bounds__(256) maxpool_bwd_s2k3_kernel(const bf16_t* __restrict__ dy,
                                                              const uint8_t* __restrict__ idx, bf16_t* __restrict__ dx,
                                                              int N, int H, int W, int C, int OH, int OW) {
  const int CT = C / 8;
  const int Hb = (H + 1) / 2, Wb = (W + 1) / 2;
  const long total = (long)N * Hb * Wb * CT;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int vc = (int)(t % CT);
    long r = t / CT;
    const int bj = (int)(r % Wb); r /= Wb;
    const int bi = (int)(r % Hb);
    const int n = (int)(r / Hb);
    float acc[2][2][8];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[a][b][j] = 0.f;
#pragma unroll
    for (int wy = 0; wy < 2; ++wy) {
      const int oh = bi + wy;
      if (oh >= OH) continue;
#pragma unroll
      for (int wx = 0; wx < 2; ++wx) {
        const int ow = bj + wx;
        if (ow >= OW) continue;
        const long oo = (((long)n * OH + oh) * OW + ow) * C + vc * 8;
        const us8 g = *reinterpret_cast<const us8*>(dy + oo);
        const uint64_t id = *reinterpret_cast<const uint64_t*>(idx + oo);
        // window origin (2oh-1, 2ow-1); input (2bi+a, 2bj+b) has tap (2bi+a-2oh+1)*3 + (2bj+b-2ow+1)
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          const int kh = a + 1 - 2 * wy;  // 2bi+a - (2(bi+wy)-1)
          if (kh < 0 || kh > 2) continue;
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const int kw = b + 1 - 2 * wx;
            if (kw < 0 || kw > 2) continue;
            const uint32_t want = (uint32_t)(kh * 3 + kw);
#pragma unroll
            for (int j = 0; j < 8; ++j)
              if (((id >> (8 * j)) & 0xff) == want) acc[a][b][j] += bf2f(g[j]);
          }
        }
      }
    }
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int h = 2 * bi + a;
      if (h >= H) continue;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int w = 2 * bj + b;
        if (w >= W) continue;
        us8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[a][b][j]);
        *reinterpret_cast<us8*>(dx + (((long)n * H + h) * W + w) * C + vc * 8) = o;
      }
    }
  }
}


// ResNet stem tail, forward: y = maxpool3x3/2/1(relu(z * scale + shift)) in one pass over
// the stem convolution output z -- the BatchNorm+ReLU output (the largest activation of
// the network, 64 ch at 112x112) is never written or re-read.  Each window element is
// rounded to bf16 before the max, exactly as the separate BN-apply + max-pool would see
// it; the 1-byte argmax per output channel feeds the backward.  ss = [scale C | shift C].
//
// The kernel is VALU-bound if written per tap (a float compare-and-select chain: ~2,000
// VALU per thread, profiles/r5_s21 0.64 ms at b1024), so the max runs on integer keys:
// after the ReLU the bf16 bit pattern orders like an unsigned integer, and
//   key = bits << 16 | (63 - (3 kh + kx))
// (kx = column in the thread's 3x5 patch) makes max(key) the window maximum AND its first
// row-major tap -- the strict '>' scan's tie rule -- in one v_max3_u32 per three taps.
// 3 kh + kx orders both windows' taps row-major (kx <= 2 for the first, 2 <= kx <= 4 for
// the second) and decodes to the tap with one subtraction.  BN + ReLU + rounding run on
// packed pairs (v_pk_fma_f32, v_cvt_pk_bf16_f32, v_pk_max_i16 against 0 on the bf16 bits).
// Border taps load the clamped (duplicate) pixel and take the duplicate's key, so they
// change neither the max nor the argmax and need no mask.
typedef float pf2 __attribute__((ext_vector_type(2)));
typedef short ps2 __attribute__((ext_vector_type(2)));
typedef __bf16 pb2 __attribute__((ext_vector_type(2)));
typedef unsigned short pu2 __attribute__((ext_vector_type(2)));

// two packed bf16 z -> two packed bf16 relu(z * s + h), rounded as f2bf would
__device__ __forceinline__ uint32_t bn_relu_pk(uint32_t p, pf2 s, pf2 h) {
  const pf2 x = {__uint_as_float(p << 16), __uint_as_float(p & 0xffff0000u)};
  const pf2 f = __builtin_elementwise_fma(x, s, h);
  const ps2 q = __builtin_bit_cast(ps2, __builtin_convertvector(f, pb2));
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(q, (ps2){0, 0}));
}

__device__ __forceinline__ uint32_t max3u(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_elementwise_max(__builtin_elementwise_max(a, b), c);
}

__global__ void __launch_bounds__(256) bn_relu_maxpool_s2k3_kernel(const bf16_t* __restrict__ z,
                                                                  const float* __restrict__ ss,
                                                                  bf16_t* __restrict__ y, uint8_t* __restrict__ idx,
                                                                  int N, int H, int W, int C, int OH, int OW) {
  // one thread: two horizontally adjacent outputs (ow, ow + 1), 8 channels -- their windows
  // share a column, so 15 loads instead of 18, all issued before any is used
  const int CT = C / 8;
  const int OW2 = (OW + 1) / 2;
  const long total = (long)N * OH * OW2 * CT;
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < (uint32_t)total; t += gridDim.x * blockDim.x) {
    const int vc = (int)(t % (uint32_t)CT);
    uint32_t r = t / (uint32_t)CT;
    const int ow0 = 2 * (int)(r % (uint32_t)OW2); r /= (uint32_t)OW2;
    const int oh = (int)(r % (uint32_t)OH);
    const int n = (int)(r / (uint32_t)OH);
    const float4 s0 = *reinterpret_cast<const float4*>(ss + vc * 8);
    const float4 s1 = *reinterpret_cast<const float4*>(ss + vc * 8 + 4);
    const float4 h0 = *reinterpret_cast<const float4*>(ss + C + vc * 8);
    const float4 h1 = *reinterpret_cast<const float4*>(ss + C + vc * 8 + 4);
    const pf2 sc[4] = {{s0.x, s0.y}, {s0.z, s0.w}, {s1.x, s1.y}, {s1.z, s1.w}};
    const pf2 sh[4] = {{h0.x, h0.y}, {h0.z, h0.w}, {h1.x, h1.y}, {h1.z, h1.w}};
    uint4 v[3][5];
    uint32_t lo[3][5];  // 63 - (3 kh + kx) of the pixel actually loaded (clamped)
    int wo[5], kxc[5];  // clamped columns: element offset in the row, patch column
#pragma unroll
    for (int kx = 0; kx < 5; ++kx) {
      const int w = ow0 * 2 - 1 + kx;
      const int wc = w < 0 ? 0 : (w >= W ? W - 1 : w);
      wo[kx] = wc * C + vc * 8;
      kxc[kx] = wc - ow0 * 2 + 1;
    }
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int h = oh * 2 - 1 + kh;
      const int hc = h < 0 ? 0 : (h >= H ? H - 1 : h);
      const bf16_t* zr = z + (long)((n * H + hc) * W) * C;
#pragma unroll
      for (int kx = 0; kx < 5; ++kx) {
        lo[kh][kx] = (uint32_t)(63 - 3 * (hc - oh * 2 + 1) - kxc[kx]);
        v[kh][kx] = *reinterpret_cast<const uint4*>(zr + wo[kx]);
      }
    }
    uint32_t best[2][8];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      uint32_t key[5][8];
#pragma unroll
      for (int kx = 0; kx < 5; ++kx) {
        const uint32_t u[4] = {v[kh][kx].x, v[kh][kx].y, v[kh][kx].z, v[kh][kx].w};
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const uint32_t b = bn_relu_pk(u[p], sc[p], sh[p]);
          key[kx][2 * p] = (b << 16) | lo[kh][kx];
          key[kx][2 * p + 1] = (b & 0xffff0000u) | lo[kh][kx];
        }
      }
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t m = max3u(key[2 * q][j], key[2 * q + 1][j], key[2 * q + 2][j]);
          best[q][j] = kh == 0 ? m : __builtin_elementwise_max(best[q][j], m);
        }
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int ow = ow0 + q;
      if (ow >= OW) continue;
      uint4 o;
      uint32_t ob[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) ob[j] = (uint32_t)(63 - 2 * q) - (best[q][j] & 63u);  // tap index
      o.x = (best[q][1] & 0xffff0000u) | (best[q][0] >> 16);
      o.y = (best[q][3] & 0xffff0000u) | (best[q][2] >> 16);
      o.z = (best[q][5] & 0xffff0000u) | (best[q][4] >> 16);
      o.w = (best[q][7] & 0xffff0000u) | (best[q][6] >> 16);
      uint2 pk;
      pk.x = ob[0] | (ob[1] << 8) | (ob[2] << 16) | (ob[3] << 24);
      pk.y = ob[4] | (ob[5] << 8) | (ob[6] << 16) | (ob[7] << 24);
      const long oo = (((long)n * OH + oh) * OW + ow) * C + vc * 8;
      *reinterpret_cast<uint4*>(y + oo) = o;
      *reinterpret_cast<uint2*>(idx + oo) = pk;
    }
  }
}

// ResNet stem tail, backward of the max-pool fused with the BatchNorm-backward statistics:
// one thread per 2x2 block of stem pixels (8 channels) as maxpool_bwd_s2k3_kernel, but a
// window's gradient is gated by its pooled output > 0 (= the ReLU derivative at its argmax
// pixel, so no ReLU mask exists), and the gated gradient g it writes is also reduced into
// per-block channel partials [sum g | sum g*z] -- the BN backward skips its statistics
// pass over g and z.  The grid is fixed (grid-stride loop); 256 % (C/8) == 0 keeps each
// thread on one channel group.
//
// WRITE_G = false: statistics only; maxpool_bwd_s2k3_bnapply_kernel then recomputes g from
// the pooled gradient (0.6 GB of dy / pooled output / argmax instead of the 1.6 GB g written
// and read back at b1024) and applies the BN backward to it -- g never reaches memory.

// g of the 2x2 stem-pixel block (bi, bj) of image n, channels 8 vc .. 8 vc + 7, rounded to
// bf16 as the stored tensor was.  Branch-free (the per-tap 'if' chain compiled to ~150 exec-mask
// branches and ~1,100 VALU per thread: profiles/r5_s21 0.65 + 0.88 ms): a window's gradient is
// gated on the packed bf16 bits -- pooled output > 0 and window inside the image, v_pk_min_u16
// to a 0/1 multiplier and v_pk_mul_lo_u16 -- then each of the block's 9 (window, pixel) pairs
// is one argmax-byte compare and select; a pixel's terms add in window order (wy, wx) as before.
__device__ __forceinline__ void stem_block_grad(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ ypool,
                                                const uint8_t* __restrict__ idx, int n, int bi, int bj, int vc,
                                                int C, int OH, int OW, float (&acc)[2][2][8]) {
  // the four windows' loads first (clamped; a clamped window's gate is zero)
  uint4 gvs[2][2], yvs[2][2];
  uint2 ids[2][2];
  const int owc[2] = {bj * C + vc * 8, (bj + 1 < OW ? bj + 1 : OW - 1) * C + vc * 8};
#pragma unroll
  for (int wy = 0; wy < 2; ++wy)
#pragma unroll
    for (int wx = 0; wx < 2; ++wx) {
      const int oh = bi + wy < OH ? bi + wy : OH - 1;
      const long oo = (long)((n * OH + oh) * OW) * C + owc[wx];
      gvs[wy][wx] = *reinterpret_cast<const uint4*>(dy + oo);
      yvs[wy][wx] = *reinterpret_cast<const uint4*>(ypool + oo);
      ids[wy][wx] = *reinterpret_cast<const uint2*>(idx + oo);
    }
  float gw[2][2][8];  // gated window gradients
  uint32_t tw[2][2][8];  // argmax taps
#pragma unroll
  for (int wy = 0; wy < 2; ++wy)
#pragma unroll
    for (int wx = 0; wx < 2; ++wx) {
      const bool inside = bi + wy < OH && bj + wx < OW;
      const pu2 lim = inside ? (pu2){1, 1} : (pu2){0, 0};
      const uint32_t gu[4] = {gvs[wy][wx].x, gvs[wy][wx].y, gvs[wy][wx].z, gvs[wy][wx].w};
      const uint32_t yu[4] = {yvs[wy][wx].x, yvs[wy][wx].y, yvs[wy][wx].z, yvs[wy][wx].w};
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        // y >= 0 (a ReLU output): bits > 0 <=> y > 0; min(bits, 1) is the 0/1 multiplier
        const pu2 mul = __builtin_elementwise_min(__builtin_bit_cast(pu2, yu[p]), lim);
        const uint32_t gg = __builtin_bit_cast(uint32_t, __builtin_bit_cast(pu2, gu[p]) * mul);
        gw[wy][wx][2 * p] = __uint_as_float(gg << 16);
        gw[wy][wx][2 * p + 1] = __uint_as_float(gg & 0xffff0000u);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) tw[wy][wx][j] = ((j < 4 ? ids[wy][wx].x : ids[wy][wx].y) >> (8 * (j & 3))) & 0xffu;
    }
  // pixel (a, b) is tap (a + 1 - 2 wy) * 3 + (b + 1 - 2 wx) of window (wy, wx) when both are in [0, 2]
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    acc[0][0][j] = tw[0][0][j] == 4 ? gw[0][0][j] : 0.f;
    acc[0][1][j] = (tw[0][0][j] == 5 ? gw[0][0][j] : 0.f) + (tw[0][1][j] == 3 ? gw[0][1][j] : 0.f);
    acc[1][0][j] = (tw[0][0][j] == 7 ? gw[0][0][j] : 0.f) + (tw[1][0][j] == 1 ? gw[1][0][j] : 0.f);
    acc[1][1][j] = (tw[0][0][j] == 8 ? gw[0][0][j] : 0.f) + (tw[0][1][j] == 6 ? gw[0][1][j] : 0.f) +
                   (tw[1][0][j] == 2 ? gw[1][0][j] : 0.f) + (tw[1][1][j] == 0 ? gw[1][1][j] : 0.f);
  }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[a][b][j] = bf2f(f2bf(acc[a][b][j]));
}

template <bool WRITE_G>
__global__ void __launch_bounds__(256) maxpool_bwd_s2k3_bnstats_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ ypool, const uint8_t* __restrict__ idx,
    const bf16_t* __restrict__ z, bf16_t* __restrict__ g, float* __restrict__ part, int N, int H, int W, int C,
    int OH, int OW) {
  __shared__ float red[256][17];
  const int CT = C / 8;
  const int Hb = (H + 1) / 2, Wb = (W + 1) / 2;
  const long total = (long)N * Hb * Wb * CT;
  float s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
  const uint32_t t0 = blockIdx.x * blockDim.x + threadIdx.x;
  for (uint32_t t = t0; t < (uint32_t)total; t += gridDim.x * blockDim.x) {
    const int vc = (int)(t % (uint32_t)CT);
    uint32_t r = t / (uint32_t)CT;
    const int bj = (int)(r % (uint32_t)Wb); r /= (uint32_t)Wb;
    const int bi = (int)(r % (uint32_t)Hb);
    const int n = (int)(r / (uint32_t)Hb);
    us8 zvs[2][2];  // z of the block, loaded up front (clamped) with the windows' operands
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int h = 2 * bi + a < H ? 2 * bi + a : H - 1, w = 2 * bj + b < W ? 2 * bj + b : W - 1;
        zvs[a][b] = *reinterpret_cast<const us8*>(z + (long)((n * H + h) * W) * C + (w * C + vc * 8));
      }
    float acc[2][2][8];
    stem_block_grad(dy, ypool, idx, n, bi, bj, vc, C, OH, OW, acc);
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int h = 2 * bi + a;
      if (h >= H) continue;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int w = 2 * bj + b;
        if (w >= W) continue;
        const long off = (long)((n * H + h) * W) * C + (w * C + vc * 8);
        const us8 zv = zvs[a][b];
        us8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          o[j] = f2bf(acc[a][b][j]);
          const float gr = acc[a][b][j];  // the stored (bf16) gradient, as the BN backward reads it
          s1[j] += gr;
          s2[j] += gr * bf2f(zv[j]);
        }
        if constexpr (WRITE_G) *reinterpret_cast<us8*>(g + off) = o;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[threadIdx.x][j] = s1[j];
    red[threadIdx.x][8 + j] = s2[j];
  }
  __syncthreads();
  // channel c = 8*vc + j lives in threads vc, vc + CT, vc + 2CT, ... of this block
  for (int c = threadIdx.x; c < 2 * C; c += blockDim.x) {
    const int k = c / C, cc = c - k * C, vc = cc >> 3, j = cc & 7;
    float tsum = 0.f;
    for (int th = vc; th < 256; th += CT) tsum += red[th][8 * k + j];
    part[(long)blockIdx.x * 2 * C + c] = tsum;
  }
}

// dz = A*g + B*z + D (bn_bwd_apply_kernel<false, false>) with g recomputed per 2x2 block
__global__ void __launch_bounds__(256) maxpool_bwd_s2k3_bnapply_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ ypool, const uint8_t* __restrict__ idx,
    const bf16_t* __restrict__ z, const float* __restrict__ coef, bf16_t* __restrict__ dz, int N, int H, int W,
    int C, int OH, int OW) {
  const int CT = C / 8;
  const int Hb = (H + 1) / 2, Wb = (W + 1) / 2;
  const long total = (long)N * Hb * Wb * CT;
  const uint32_t t0 = blockIdx.x * blockDim.x + threadIdx.x;
  for (uint32_t t = t0; t < (uint32_t)total; t += gridDim.x * blockDim.x) {
    const int vc = (int)(t % (uint32_t)CT);
    uint32_t r = t / (uint32_t)CT;
    const int bj = (int)(r % (uint32_t)Wb); r /= (uint32_t)Wb;
    const int bi = (int)(r % (uint32_t)Hb);
    const int n = (int)(r / (uint32_t)Hb);
    float A[8], B[8], D[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      A[j] = coef[vc * 8 + j];
      B[j] = coef[C + vc * 8 + j];
      D[j] = coef[2 * C + vc * 8 + j];
    }
    float acc[2][2][8];
    stem_block_grad(dy, ypool, idx, n, bi, bj, vc, C, OH, OW, acc);
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int h = 2 * bi + a;
      if (h >= H) continue;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int w = 2 * bj + b;
        if (w >= W) continue;
        const long off = (long)((n * H + h) * W) * C + (w * C + vc * 8);
        const us8 zv = *reinterpret_cast<const us8*>(z + off);
        us8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf(bn_bwd_affine(A[j], acc[a][b][j], B[j], bf2f(zv[j]), D[j]));
        *reinterpret_cast<us8*>(dz + off) = o;
      }
    }
  }
}

extern "C" {

int ca_bn_relu_maxpool_s2k3(const bf16_t* z, const float* ss, bf16_t* y, uint8_t* idx, int N, int H, int W, int C,
                            int OH, int OW, hipStream_t st) {
  if (C % 8 != 0 || OH != (H - 1) / 2 + 1 || OW != (W - 1) / 2 + 1) return -1;
  const long total = (long)N * OH * ((OW + 1) / 2) * (C / 8);
  if (total >= (1L << 31) || (long)N * H * W >= (1L << 31)) return -1;  // 32-bit thread / pixel indices
  const int grid = (int)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
  bn_relu_maxpool_s2k3_kernel<<<grid, 256, 0, st>>>(z, ss, y, idx, N, H, W, C, OH, OW);
  CA_LAUNCH_CHECK();
  return 0;
}

// blocks of the fixed grid (= rows of the partials) ca_maxpool_bwd_s2k3_bnstats uses
int ca_maxpool_bnstats_parts(int N, int H, int W, int C) {
  const long total = (long)N * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8);
  const long b = (total + 255) / 256;
  return (int)(b < 1024 ? b : 1024);
}

int ca_maxpool_bwd_s2k3_bnstats(const bf16_t* dy, const bf16_t* ypool, const uint8_t* idx, const bf16_t* z, bf16_t* g,
                                float* part, int N, int H, int W, int C, int OH, int OW, hipStream_t st) {
  if (C % 8 != 0 || 256 % (C / 8) != 0 || OH != (H - 1) / 2 + 1 || OW != (W - 1) / 2 + 1) return -1;
  if ((long)N * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8) >= (1L << 31) || (long)N * H * W >= (1L << 31))
    return -1;  // 32-bit thread / pixel indices
  const int grid = ca_maxpool_bnstats_parts(N, H, W, C);
  if (g) maxpool_bwd_s2k3_bnstats_kernel<true><<<grid, 256, 0, st>>>(dy, ypool, idx, z, g, part, N, H, W, C, OH, OW);
  else maxpool_bwd_s2k3_bnstats_kernel<false><<<grid, 256, 0, st>>>(dy, ypool, idx, z, g, part, N, H, W, C, OH, OW);
  CA_LAUNCH_CHECK();
  return 0;
}

// dz[N,H,W,C] = the BN backward (coef = [A | B | D] from the statistics finalize) of the stem
// max-pool gradient, recomputed from the pooled gradient / output / argmax (see above).
int ca_maxpool_bwd_s2k3_bnapply(const bf16_t* dy, const bf16_t* ypool, const uint8_t* idx, const bf16_t* z,
                                const float* coef, bf16_t* dz, int N, int H, int W, int C, int OH, int OW,
                                hipStream_t st) {
  if (C % 8 != 0 || OH != (H - 1) / 2 + 1 || OW != (W - 1) / 2 + 1) return -1;
  const long total = (long)N * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8);
  if (total >= (1L << 31) || (long)N * H * W >= (1L << 31)) return -1;  // 32-bit thread / pixel indices
  maxpool_bwd_s2k3_bnapply_kernel<<<ca_stream_grid(total, 256), 256, 0, st>>>(dy, ypool, idx, z, coef, dz, N, H, W,
                                                                              C, OH, OW);
  CA_LAUNCH_CHECK();
  return 0;
}


int ca_stem_s2d(const bf16_t* x, bf16_t* y, int N, int H, int W, int C, int Hs, int Ws, int pad, hipStream_t st) {
  if (C < 1 || C > 4) return -1;
  const long total = (long)N * Hs * Ws;
  stem_s2d_kernel<<<(unsigned)((total + 255) / 256), 256, 0, st>>>(x, y, N, H, W, C, Hs, Ws, pad);
  CA_LAUNCH_CHECK();
  return 0;
}

int ca_maxpool_fwd(const bf16_t* x, bf16_t* y, uint8_t* idx, int N, int H, int W, int C, int OH, int OW,
                   int k, int s, int p, hipStream_t st) {
  if (C % 8 || k * k > 255) return -1;
  const long total = (long)N * OH * OW * (C / 8);
  maxpool_fwd_kernel<<<ca_stream_grid(total, 256), 256, 0, st>>>(x, y, idx, N, H, W, C, OH, OW, k, s, p);
  CA_LAUNCH_CHECK();
  return 0;
}

int ca_maxpool_bwd(const bf16_t* dy, const uint8_t* idx, bf16_t* dx, int N, int H, int W, int C, int OH, int OW,
                   int k, int s, int p, hipStream_t st) {
  if (C % 8) return -1;
  const long total = (long)N * H * W * (C / 8);
  if (k == 3 && s == 2 && p == 1 && OH == (H - 1) / 2 + 1 && OW == (W - 1) / 2 + 1) {
    const long blocks = (long)N * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8);
    maxpool_bwd_s2k3_kernel<<<ca_stream_grid(blocks, 256), 256, 0, st>>>(dy, idx, dx, N, H, W, C, OH, OW);
    CA_LAUNCH_CHECK();
    return 0;
  }
  maxpool_bwd_kernel<<<ca_stream_grid(total, 256), 256, 0, st>>>(dy, idx, dx, N, H, W, C, OH, OW, k, s, p);
  CA_LAUNCH_CHECK();
  return 0;
}

int ca_gap_fwd(const bf16_t* x, void* y, int y_is_bf16, int N, int HW, int C, hipStream_t st) {
  if (C % 8) return -1;
  const long total = (long)N * (C / 8);
  if (y_is_bf16) gap_fwd_kernel<bf16_t><<<ca_stream_grid(total, 256), 256, 0, st>>>(x, (bf16_t*)y, N, HW, C);
  else gap_fwd_kernel<float><<<ca_stream_grid(total, 256), 256, 0, st>>>(x, (float*)y, N, HW, C);
  CA_LAUNCH_CHECK();
  return 0;
}

int ca_gmp_fwd(const bf16_t* x, bf16_t* y, float* cnt, int N, int HW, int C, hipStream_t st) {
  if (C % 8) return -1;
  const long total = (long)N * (C / 8);
  gmp_fwd_kernel<<<ca_stream_grid(total, 256), 256, 0, st>>>(x, y, cnt, N, HW, C);
  CA_LAUNCH_CHECK();
  return 0;
}

int ca_gmp_bwd(const void* dy, int dy_is_bf16, const bf16_t* x, const bf16_t* y, const float* cnt, bf16_t* dx, int N,
               int HW, int C, hipStream_t st) {
  if (C % 8) return -1;
  const long total = (long)N * HW * (C / 8);
  if (dy_is_bf16)
    gmp_bwd_kernel<bf16_t><<<ca_stream_grid(total, 256), 256, 0, st>>>((const bf16_t*)dy, x, y, cnt, dx, N, HW, C);
  else
    gmp_bwd_kernel<float><<<ca_stream_grid(total, 256), 256, 0, st>>>((const float*)dy, x, y, cnt, dx, N, HW, C);
  CA_LAUNCH_CHECK();
  return 0;
}

int ca_gap_bwd(const void* dy, int dy_is_bf16, bf16_t* dx, int N, int HW, int C, hipStream_t st) {
  if (C % 8) return -1;
  const long total = (long)N * HW * (C / 8);
  if (dy_is_bf16) gap_bwd_kernel<bf16_t><<<ca_stream_grid(total, 256), 256, 0, st>>>((const bf16_t*)dy, dx, N, HW, C);
  else gap_bwd_kernel<float><<<ca_stream_grid(total, 256), 256, 0, st>>>((const float*)dy, dx, N, HW, C);
  CA_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
