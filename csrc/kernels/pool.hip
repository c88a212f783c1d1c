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
__global__ void __launch_bounds__(256) bn_relu_maxpool_s2k3_kernel(const bf16_t* __restrict__ z,
                                                                  const float* __restrict__ ss,
                                                                  bf16_t* __restrict__ y, uint8_t* __restrict__ idx,
                                                                  int N, int H, int W, int C, int OH, int OW) {
  // one thread: two horizontally adjacent outputs (ow, ow + 1), 8 channels -- their windows
  // share a column, so 15 loads instead of 18, all issued before any is used (clamped
  // addresses, border taps masked after)
  const int CT = C / 8;
  const int OW2 = (OW + 1) / 2;
  const long total = (long)N * OH * OW2 * CT;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int vc = (int)(t % CT);
    long r = t / CT;
    const int ow0 = 2 * (int)(r % OW2); r /= OW2;
    const int oh = (int)(r % OH);
    const int n = (int)(r / OH);
    float sc[8], sh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sc[j] = ss[vc * 8 + j];
      sh[j] = ss[C + vc * 8 + j];
    }
    us8 v[3][5];
    bool ok[3][5];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int h = oh * 2 - 1 + kh;
      const int hc = h < 0 ? 0 : (h >= H ? H - 1 : h);
#pragma unroll
      for (int kx = 0; kx < 5; ++kx) {
        const int w = ow0 * 2 - 1 + kx;
        const int wc = w < 0 ? 0 : (w >= W ? W - 1 : w);
        ok[kh][kx] = h >= 0 && h < H && w >= 0 && w < W;
        v[kh][kx] = *reinterpret_cast<const us8*>(z + (((long)n * H + hc) * W + wc) * C + vc * 8);
      }
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int ow = ow0 + q;
      if (ow >= OW) continue;
      float best[8];
      uint8_t bi[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        best[j] = -INFINITY;
        bi[j] = 0;
      }
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int kx = 2 * q + kw;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float f = fmaxf(bf2f(v[kh][kx][j]) * sc[j] + sh[j], 0.f);
            f = bf2f(f2bf(f));
            if (ok[kh][kx] && f > best[j]) { best[j] = f; bi[j] = (uint8_t)(kh * 3 + kw); }
          }
        }
      }
      us8 o;
      uint64_t packed = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o[j] = f2bf(best[j]);
        packed |= (uint64_t)bi[j] << (8 * j);
      }
      const long oo = (((long)n * OH + oh) * OW + ow) * C + vc * 8;
      *reinterpret_cast<us8*>(y + oo) = o;
      *reinterpret_cast<uint64_t*>(idx + oo) = packed;
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
// bf16 as the stored tensor was
__device__ __forceinline__ void stem_block_grad(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ ypool,
                                                const uint8_t* __restrict__ idx, int n, int bi, int bj, int vc,
                                                int C, int OH, int OW, float (&acc)[2][2][8]) {
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[a][b][j] = 0.f;
  // the four windows' loads first (clamped, masked after): none behind a branch
  us8 gvs[2][2], yvs[2][2];
  uint64_t ids[2][2];
#pragma unroll
  for (int wy = 0; wy < 2; ++wy)
#pragma unroll
    for (int wx = 0; wx < 2; ++wx) {
      const int oh = bi + wy < OH ? bi + wy : OH - 1, ow = bj + wx < OW ? bj + wx : OW - 1;
      const long oo = (((long)n * OH + oh) * OW + ow) * C + vc * 8;
      gvs[wy][wx] = *reinterpret_cast<const us8*>(dy + oo);
      yvs[wy][wx] = *reinterpret_cast<const us8*>(ypool + oo);
      ids[wy][wx] = *reinterpret_cast<const uint64_t*>(idx + oo);
    }
#pragma unroll
  for (int wy = 0; wy < 2; ++wy) {
    const int oh = bi + wy;
    if (oh >= OH) continue;
#pragma unroll
    for (int wx = 0; wx < 2; ++wx) {
      const int ow = bj + wx;
      if (ow >= OW) continue;
      const us8 gv = gvs[wy][wx];
      const us8 yv = yvs[wy][wx];
      const uint64_t id = ids[wy][wx];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int kh = a + 1 - 2 * wy;
        if (kh < 0 || kh > 2) continue;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const int kw = b + 1 - 2 * wx;
          if (kw < 0 || kw > 2) continue;
          const uint32_t want = (uint32_t)(kh * 3 + kw);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (((id >> (8 * j)) & 0xff) == want && bf2f(yv[j]) > 0.f) acc[a][b][j] += bf2f(gv[j]);
        }
      }
    }
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
  const long t0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (long t = t0; t < total; t += (long)gridDim.x * blockDim.x) {
    const int vc = (int)(t % CT);
    long r = t / CT;
    const int bj = (int)(r % Wb); r /= Wb;
    const int bi = (int)(r % Hb);
    const int n = (int)(r / Hb);
    us8 zvs[2][2];  // z of the block, loaded up front (clamped) with the windows' operands
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int h = 2 * bi + a < H ? 2 * bi + a : H - 1, w = 2 * bj + b < W ? 2 * bj + b : W - 1;
        zvs[a][b] = *reinterpret_cast<const us8*>(z + (((long)n * H + h) * W + w) * C + vc * 8);
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
        const long off = (((long)n * H + h) * W + w) * C + vc * 8;
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
  const long t0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (long t = t0; t < total; t += (long)gridDim.x * blockDim.x) {
    const int vc = (int)(t % CT);
    long r = t / CT;
    const int bj = (int)(r % Wb); r /= Wb;
    const int bi = (int)(r % Hb);
    const int n = (int)(r / Hb);
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
        const long off = (((long)n * H + h) * W + w) * C + vc * 8;
        const us8 zv = *reinterpret_cast<const us8*>(z + off);
        us8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf(A[j] * acc[a][b][j] + B[j] * bf2f(zv[j]) + D[j]);
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
