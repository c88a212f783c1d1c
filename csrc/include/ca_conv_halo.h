// 3x3 / stride-1 / pad-1 convolution over 64 channels with the input patch and the weights
// resident in LDS (gfx950 / CDNA4) -- ResNet-50's stage-1 conv2 forward and its input gradient.
//
// The implicit-GEMM kernels (conv.hip, GConvFwdAT / GConvDgradAT loaders) gather every K tile
// of a 3x3 convolution from global memory: each input pixel is fetched through L2 nine times,
// and with 64 channels a 256 x 64 output tile runs only 9 K tiles, so the pipeline fill and the
// epilogue are a large share of every tile (stage 1 ran at 440-660 TF/s against 900-1,100 for
// stages 2-4, docs/performance.md).  Here a persistent workgroup (one per CU, 7 waves)
//
//   * keeps the whole 3x3 x 64 x 64 filter in LDS for its lifetime (73,728 B, written once),
//   * walks tiles of 8 output rows x the full image width W (= 56: 448 pixels = 7 waves x 64),
//   * stages each tile's input patch -- 10 rows x (W + 2) columns x 64 channels, zero borders --
//     ONCE into LDS (74,240 B): the nine taps are nine shifted views of it, read with
//     ds_read_b128 (no tap is gathered from global memory),
//   * loads the NEXT tile's patch into registers (10 x 16 B per thread) while the MFMAs of the
//     current one run, and writes it to LDS behind the tile's last barrier,
//   * multiplies with v_mfma_f32_16x16x32_bf16: wave w owns pixels [64 w, 64 w + 64) of the tile
//     and all 64 output channels (4 x 4 fragments), K = 9 taps x 64 channels = 18 steps of 32,
//   * and accumulates the BatchNorm statistics of everything it stores in registers across all
//     its tiles, writing ONE [2][64] partial row per workgroup (the consumer sums the rows).
//
// Input gradient (dgrad = 1): dX = conv(dY, W') with W'[ci][kh][kw][co] = W[co][2-kh][2-kw][ci]
// -- the same kernel over a rotated, transposed filter image, with the BN-backward statistics
// epilogue of conv.hip (sum g, sum g * z, g = dX gated by the ReLU bitmask of the BN that
// produced the conv's input).
//
// LDS images are [row][64 channels] (128 B per row); 16-B chunk c of row q is stored at chunk
// c ^ ((q >> 1) & 7), so the 16 lanes of a ds_read_b128 lane group, which read 16 consecutive
// rows at one chunk, hit 16 distinct 16-B bank slots (two rows share a 256-B bank row).
#pragma once
#include "ca_mfma_core.h"

namespace ca {

struct HaloParams {
  const bf16_t* x;        // input [N][H][W][64] (dgrad: dY)
  const bf16_t* w;        // filter [64][3][3][64] (OHWI)
  bf16_t* y;              // output [N][H][W][64] (dgrad: dX)
  float* stats;           // [gridDim.x][2][64]: [sum | sum of squares] (fwd) or [sum g | sum g*z] (dgrad)
  const bf16_t* bnz;      // dgrad statistics: BN input z [N][H][W][64]
  const uint8_t* bnmask;  // dgrad statistics: ReLU bitmask [N*H*W][8]
  int N, H, W;
  int dgrad;
};

constexpr int HALO_C = 64, HALO_TR = 8, HALO_WAVES = 7, HALO_NT = HALO_WAVES * 64;

__device__ __forceinline__ int halo_swz(int q, int chunk) { return q * 64 + ((chunk ^ ((q >> 1) & 7)) << 3); }

// W = 56 only (8 x 56 = 448 = 7 x 64 pixels per tile); H % 8 == 0 (host-checked).
template <bool STATS>
__device__ __forceinline__ void conv3x3_halo(const HaloParams& P) {
  constexpr int C = HALO_C, TR = HALO_TR, NT = HALO_NT, W = 56, PW = W + 2, PR = TR + 2;
  constexpr int WIMG = 9 * C * C;      // shorts
  constexpr int PIMG = PR * PW * C;    // shorts
  constexpr int PCH = PR * W * 8;      // 16-B chunks of a patch's interior = 4480 = 10 per thread
  static_assert(PCH % NT == 0, "patch chunks must divide the threads");
  constexpr int PPT = PCH / NT;
  constexpr int SRED = STATS ? HALO_WAVES * 2 * C * 2 : 0;  // shorts: per-wave [2][64] fp32 statistics
  __shared__ __attribute__((aligned(16))) short smem[WIMG + PIMG + SRED];
  short* wimg = smem;
  short* pimg = smem + WIMG;
  float* sred = reinterpret_cast<float*>(smem + WIMG + PIMG);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = P.H;
  const int rgroups = H / TR;
  const int ntiles = P.N * rgroups;

  // filter image [tap][n][k]: fwd n = co, k = ci (W[co][tap][ci]); dgrad n = ci, k = co
  // (W[co][8 - tap][ci]).  Written once.
  for (int e = tid; e < 9 * C * 8; e += NT) {
    const int tap = e / (C * 8), n = (e / 8) % C, ch = e % 8;
    s8v v;
    if (!P.dgrad) {
      v = *reinterpret_cast<const s8v*>(P.w + ((long)n * 9 + tap) * C + ch * 8);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (short)P.w[((long)(ch * 8 + j) * 9 + (8 - tap)) * C + n];
    }
    *reinterpret_cast<s8v*>(wimg + halo_swz(tap * C + n, ch)) = v;
  }
  // the patch's left / right zero columns never change
  for (int e = tid; e < PR * 2 * 8; e += NT) {
    const int r = e / 16, side = (e / 8) & 1, ch = e % 8;
    *reinterpret_cast<s8v*>(pimg + halo_swz(r * PW + (side ? PW - 1 : 0), ch)) = zero8();
  }

  // this thread's patch chunks: interior chunk e = (r, c, ch), r in [0, PR), c in [0, W)
  auto load_patch = [&](int t, s8v (&v)[PPT]) {
    const int n = t / rgroups, r0 = (t % rgroups) * TR - 1;  // patch row 0 = image row r0
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int e = tid + i * NT;
      const int r = e / (W * 8), c = (e / 8) % W, ch = e % 8;
      const int ir = r0 + r;
      v[i] = (ir >= 0 && ir < H) ? *reinterpret_cast<const s8v*>(P.x + (((long)n * H + ir) * W + c) * C + ch * 8)
                                 : zero8();
    }
  };
  auto store_patch = [&](const s8v (&v)[PPT]) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int e = tid + i * NT;
      const int r = e / (W * 8), c = (e / 8) % W, ch = e % 8;
      *reinterpret_cast<s8v*>(pimg + halo_swz(r * PW + c + 1, ch)) = v[i];
    }
  };

  // per lane: patch row q0 (tap (0,0)) of the pixel of each of its 4 M fragments
  int q0[4];
#pragma unroll
  for (int mf = 0; mf < 4; ++mf) {
    const int p = wave * 64 + mf * 16 + (lane & 15);
    q0[mf] = (p / W) * PW + (p % W);
  }
  const int kq = lane >> 4;  // this lane's 8-channel chunk within a 32-deep K step

  if constexpr (STATS) {
    for (int e = tid; e < HALO_WAVES * 2 * C; e += NT) sred[e] = 0.f;
  }

  int t = blockIdx.x;
  s8v nxt[PPT];
  if (t < ntiles) load_patch(t, nxt);
  for (; t < ntiles; t += gridDim.x) {
    __syncthreads();  // previous tile's LDS reads retired (and, first trip, the filter image written)
    store_patch(nxt);
    __syncthreads();
    const int tn = t + gridDim.x;
    if (tn < ntiles) load_patch(tn, nxt);  // in flight during the MFMAs below

    f4v acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
      const int dq = (tap / 3) * PW + (tap % 3);
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        const int chunk = kh * 4 + kq;
        bf16x8 af[4], bfr[4];
#pragma unroll
        for (int nf = 0; nf < 4; ++nf)
          bfr[nf] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const s8v*>(
                                                  wimg + halo_swz(tap * C + nf * 16 + (lane & 15), chunk)));
#pragma unroll
        for (int mf = 0; mf < 4; ++mf)
          af[mf] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const s8v*>(pimg + halo_swz(q0[mf] + dq, chunk)));
#pragma unroll
        for (int mf = 0; mf < 4; ++mf)
#pragma unroll
          for (int nf = 0; nf < 4; ++nf)
            acc[mf][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[nf], af[mf], acc[mf][nf], 0, 0, 0);
      }
    }

    // epilogue: lane holds pixel (mf*16 + lane&15), channels nf*16 + 4*kq + r.  The tile's
    // statistics (of channels nf * 16 + 4 * kq + r, index nf * 4 + r) are reduced over the 16
    // pixel lanes and added to this wave's LDS row, so they hold no registers across tiles.
    float ssum[16], ssq[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) ssum[j] = ssq[j] = 0.f;
    const int n = t / rgroups, r0 = (t % rgroups) * TR;
#pragma unroll
    for (int mf = 0; mf < 4; ++mf) {
      const int p = wave * 64 + mf * 16 + (lane & 15);
      const long pix = ((long)n * H + r0 + p / W) * W + (p % W);
      uint32_t mk = 0xffffffffu;
      if (STATS && P.dgrad) {
        // the 16 channels of this lane (4 groups of 4 at nf * 16 + 4 * kq) span bytes nf*2 + kq/2
        mk = 0;
        if (P.bnmask) {
#pragma unroll
          for (int nf = 0; nf < 4; ++nf)
            mk |= (((uint32_t)P.bnmask[pix * 8 + nf * 2 + (kq >> 1)] >> ((kq & 1) * 4)) & 0xfu) << (nf * 4);
        } else {
          mk = 0xffffu;
        }
      }
#pragma unroll
      for (int nf = 0; nf < 4; ++nf) {
        const int co = nf * 16 + 4 * kq;
        us4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = f2bf(acc[mf][nf][r]);
        *reinterpret_cast<us4*>(P.y + pix * C + co) = o;
        if constexpr (STATS) {
          if (!P.dgrad) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float a = bf2f(o[r]);
              ssum[nf * 4 + r] += a;
              ssq[nf * 4 + r] += a * a;
            }
          } else {
            const us4 z = *reinterpret_cast<const us4*>(P.bnz + pix * C + co);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float g = ((mk >> (nf * 4 + r)) & 1u) ? bf2f(o[r]) : 0.f;
              ssum[nf * 4 + r] += g;
              ssq[nf * 4 + r] += g * bf2f(z[r]);
            }
          }
        }
      }
    }
    if constexpr (STATS) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          ssum[j] += __shfl_xor(ssum[j], o, 64);
          ssq[j] += __shfl_xor(ssq[j], o, 64);
        }
      }
      if ((lane & 15) == 0) {  // this wave's row only: no other wave writes it
#pragma unroll
        for (int nf = 0; nf < 4; ++nf)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            sred[(wave * 2 + 0) * C + nf * 16 + 4 * kq + r] += ssum[nf * 4 + r];
            sred[(wave * 2 + 1) * C + nf * 16 + 4 * kq + r] += ssq[nf * 4 + r];
          }
      }
    }
  }
  if constexpr (STATS) {
    __syncthreads();
    if (tid < 2 * C) {
      const int k = tid / C, c = tid % C;
      float a = 0.f;
#pragma unroll
      for (int w = 0; w < HALO_WAVES; ++w) a += sred[(w * 2 + k) * C + c];
      P.stats[((long)blockIdx.x * 2 + k) * C + c] = a;
    }
  }
}

}  // namespace ca
