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
    if (idx) {
#pragma unroll
      for (int j = 0; j < 8; ++j) idx[oo + j] = bi[j];
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

extern "C" {

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

int ca_gap_bwd(const void* dy, int dy_is_bf16, bf16_t* dx, int N, int HW, int C, hipStream_t st) {
  if (C % 8) return -1;
  const long total = (long)N * HW * (C / 8);
  if (dy_is_bf16) gap_bwd_kernel<bf16_t><<<ca_stream_grid(total, 256), 256, 0, st>>>((const bf16_t*)dy, dx, N, HW, C);
  else gap_bwd_kernel<float><<<ca_stream_grid(total, 256), 256, 0, st>>>((const float*)dy, dx, N, HW, C);
  CA_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
