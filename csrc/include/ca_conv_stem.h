// ResNet stem convolution with the input patch and the filter resident in LDS (gfx950 / CDNA4):
// the 7x7 / stride-2 stem run as a 4x4 / stride-1 / unpadded convolution over the 16-channel
// space-to-depth input (conv.hip stem path, ops/conv.py _StemS2DFn), forward with the
// BatchNorm-statistics epilogue.
//
// The implicit-GEMM form (conv.hip GConvRowA on 256 x 64 tiles) reads each K tile of every
// output pixel from L2: every input pixel is fetched by the 16 output pixels whose 4 x 4 window
// covers it, ~6.5 GB of L2 reads for a 433-MB input at batch 1024, and a 256 x 64 tile runs only
// four K tiles, so its prologue and epilogue dominate (0.74 ms, 2.8 TB/s of HBM bytes moved;
// docs/performance.md, round 5 "Where the remaining time is").  Here a persistent workgroup
// (7 waves, one per CU)
//
//   * keeps the whole [64 co][256 k] filter in LDS for its lifetime (33 KB, written once; rows
//     padded to 528 B so the 16 rows a B-fragment read touches land in 16 distinct bank slots),
//   * walks tiles of TR = 4 output rows x the full width 112 (448 pixels = 7 waves x 64),
//   * stages each tile's input patch -- 7 rows x 115 pixels x 16 channels, one CONTIGUOUS
//     25,760-B run of the space-to-depth tensor -- ONCE into LDS: the 16 taps are shifted reads
//     of it.  CHUNK-MAJOR image, two planes (channels 0-7 / 8-15) of 16-B pixels: the 16 lanes
//     of an A-fragment read take 16 consecutive pixels of one plane (256 contiguous bytes,
//     conflict-free); the planes are 128 B apart modulo 256 so the staging stores of a lane
//     octet (alternating planes, consecutive pixels) are conflict-free too,
//   * loads the NEXT tile's patch into registers (4 x 16 B per thread) while the MFMAs of the
//     current one run, and writes it to LDS behind the tile's barriers,
//   * multiplies with v_mfma_f32_16x16x32_bf16: wave w owns pixels [64 w, 64 w + 64) of the
//     tile (four 16-pixel fragments, each inside one output row since 112 = 7 x 16) and all 64
//     output channels; K = 16 taps x 16 channels = 8 steps of 32 (two taps of one filter row
//     per step), the next step's fragments read during this step's MFMAs,
//   * and accumulates the BN statistics of what it stores across all its tiles, writing ONE
//     [2][64] partial row per workgroup (the stem tail sums the rows).
//
// Measured at b1024 (profiles/r6_s9..r6_s11): 0.743 ms (implicit GEMM) -> 0.626 ms; 0.609 ms with
// the counted-wait tile loop.  Not kept: 8 waves x one output row each (TR = 8, seven fragments
// per wave: 252 VGPRs, room for one fragment register set only) -- 0.749 ms.
#pragma once
#include "ca_conv_halo.h"

namespace ca {

struct StemParams {
  const bf16_t* x;  // space-to-depth input [N][OH + 3][OW + 3][16]
  const bf16_t* w;  // filter [64][4][4][16] (OHWI)
  bf16_t* y;        // output [N][OH][OW][64]
  float* stats;     // [gridDim.x][2][64]: [sum | sum of squares] of the stored bf16 values, or null
  int N, OH;        // OW = 112, OH % 4 == 0 (host-checked)
};

constexpr int STEM_C = 64, STEM_CI = 16, STEM_TR = 4, STEM_OW = 112, STEM_WAVES = 7, STEM_NT = STEM_WAVES * 64;
constexpr int STEM_PW = STEM_OW + 3, STEM_PR = STEM_TR + 3;       // patch: 7 rows x 115 pixels
constexpr int STEM_PLANE = 51 * 256 + 128;                       // bytes: >= 7 x 115 x 16, == 128 mod 256
constexpr int STEM_PCH = STEM_PR * STEM_PW * 2;                  // 16-B chunks of a patch = 1,610
constexpr int STEM_PPT = (STEM_PCH + STEM_NT - 1) / STEM_NT;     // 4 per thread (the last partial)

// filter image row co: 256 k + 8 pad shorts (528 B): the 16 rows of a B-fragment read start in
// 16 distinct 16-B bank slots, and a K step's chunk is a constant offset from the lane's row
// (an XOR swizzle of the chunk index would need one address register per step)
constexpr int STEM_WLD = 264;
__device__ __forceinline__ int stem_widx(int co, int chunk) { return co * STEM_WLD + (chunk << 3); }

template <bool STATS>
__device__ __forceinline__ void conv_stem_s2d(const StemParams& P) {
  constexpr int C = STEM_C, TR = STEM_TR, NT = STEM_NT, OW = STEM_OW, PW = STEM_PW, PPT = STEM_PPT;
  constexpr int WIMG = C * STEM_WLD;               // shorts
  constexpr int PIMG = 2 * STEM_PLANE / 2;         // shorts
  constexpr int SRED = STATS ? STEM_WAVES * 2 * C * 2 : 0;
  static_assert(STEM_PR * PW * 16 <= STEM_PLANE, "patch plane");
  __shared__ __attribute__((aligned(16))) short smem[WIMG + PIMG + SRED];
  short* wimg = smem;
  short* pimg = smem + WIMG;
  float* sred = reinterpret_cast<float*>(smem + WIMG + PIMG);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rgroups = P.OH / TR;
  const int ntiles = P.N * rgroups;
  const long img = (long)(P.OH + 3) * PW * STEM_CI;  // input elements per image

  // filter image: 64 rows of 32 16-B chunks (the OHWI row is already k-contiguous)
  for (int e = tid; e < C * 32; e += NT) {
    const int co = e >> 5, ch = e & 31;
    *reinterpret_cast<s8v*>(wimg + stem_widx(co, ch)) = *reinterpret_cast<const s8v*>(P.w + (long)co * 256 + ch * 8);
  }
  if constexpr (STATS) {
    for (int e = tid; e < STEM_WAVES * 2 * C; e += NT) sred[e] = 0.f;
  }

  // patch chunk e = tid + i * NT: pixel e >> 1 of the contiguous 7-row run, channel half e & 1.
  // Branch-free: a chunk past the patch reloads the last one (never stored) -- a load under a
  // branch makes hipcc wait vmcnt(0) where the branches join (cdna_hip_programming.md 5, item 4c).
  auto load_patch = [&](int t, s8v (&v)[PPT]) {
    const int n = t / rgroups, r0 = (t % rgroups) * TR;
    const bf16_t* src = P.x + n * img + (long)r0 * PW * STEM_CI;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int e = tid + i * NT;
      v[i] = *reinterpret_cast<const s8v*>(src + (e < STEM_PCH ? e : STEM_PCH - 1) * 8);
    }
  };
  auto store_patch = [&](const s8v (&v)[PPT]) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int e = tid + i * NT;
      if (e < STEM_PCH) *reinterpret_cast<s8v*>(pimg + (e & 1) * (STEM_PLANE / 2) + (e >> 1) * 8) = v[i];
    }
  };

  // per lane: patch pixel of tap (0, 0) for each of its 4 M fragments
  constexpr int MF = 4;
  int q0[MF];
#pragma unroll
  for (int mf = 0; mf < MF; ++mf) {
    const int p = wave * 64 + mf * 16 + (lane & 15);
    q0[mf] = (p / OW) * PW + (p % OW);
  }
  const int kq = lane >> 4;  // 8-element K chunk of the 32-deep step: tap + (kq >> 1), half kq & 1

  // Tile loop.  The next tile's patch loads are issued at the top of a tile, BEFORE its 16
  // epilogue stores, and written to LDS at the bottom behind a counted vmcnt(16): the stores stay
  // in flight across the next tile's MFMAs.  (A __syncthreads() at the top of the loop made hipcc
  // drain vmcnt to 0 there, exposing every tile's store latency: 0.63 ms for the stem at b1024.)
  // Only LDS is shared between the waves inside the loop, so raw s_barriers with lgkmcnt(0).
  int t = blockIdx.x;
  s8v nxt[PPT];
  if (t < ntiles) {
    load_patch(t, nxt);
    halo_vm_wait0();
    store_patch(nxt);
  }
  __syncthreads();  // the filter image and the first patch written
  for (; t < ntiles; t += gridDim.x) {
    const int tn = t + gridDim.x;
    load_patch(tn < ntiles ? tn : t, nxt);  // in flight during the MFMAs and stores below

    f4v acc[MF][4];
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
    const int n = t / rgroups, r0 = (t % rgroups) * TR;
    const long pix0 = ((long)n * P.OH + r0) * OW + wave * 64 + (lane & 15);  // fragment 0's pixel

    // step st: filter row kh = st >> 1, taps kw0 = 2 (st & 1) and kw0 + 1
    auto frag_load = [&](int st, bf16x8 (&af)[MF], bf16x8 (&bfr)[4]) {
      const int dq = (st >> 1) * PW + (st & 1) * 2 + (kq >> 1);
      const short* plane = pimg + (kq & 1) * (STEM_PLANE / 2);
#pragma unroll
      for (int nf = 0; nf < 4; ++nf)
        bfr[nf] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const s8v*>(
                                                 wimg + stem_widx(nf * 16 + (lane & 15), st * 4 + kq)));
#pragma unroll
      for (int mf = 0; mf < MF; ++mf)
        af[mf] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const s8v*>(plane + (q0[mf] + dq) * 8));
    };
    // the next step's fragments are read while this step's 16 MFMAs run (two register sets)
    bf16x8 fa[2][MF], fb[2][4];
    frag_load(0, fa[0], fb[0]);
#pragma unroll
    for (int st = 0; st < 8; ++st) {
      if (st + 1 < 8) frag_load(st + 1, fa[(st + 1) & 1], fb[(st + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);  // the next step's reads ahead of this step's MFMAs
#pragma unroll
      for (int mf = 0; mf < MF; ++mf)
#pragma unroll
        for (int nf = 0; nf < 4; ++nf)
          acc[mf][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[st & 1][nf], fa[st & 1][mf], acc[mf][nf], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }

    // epilogue: lane holds pixel mf*16 + (lane & 15), channels nf*16 + 4*kq + r
    float ssum[16], ssq[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) ssum[j] = ssq[j] = 0.f;
#pragma unroll
    for (int mf = 0; mf < MF; ++mf) {
      bf16_t* yp = P.y + (pix0 + mf * 16) * C + 4 * kq;
#pragma unroll
      for (int nf = 0; nf < 4; ++nf) {
        us4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = f2bf(acc[mf][nf][r]);
        *reinterpret_cast<us4*>(yp + nf * 16) = o;
        if constexpr (STATS) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float a = bf2f(o[r]);
            ssum[nf * 4 + r] += a;
            ssq[nf * 4 + r] += a * a;
          }
        }
      }
    }
    if constexpr (STATS) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        ssum[j] = row16_sum(ssum[j]);
        ssq[j] = row16_sum(ssq[j]);
      }
      if ((lane & 15) == 0) {  // this wave's row only
#pragma unroll
        for (int nf = 0; nf < 4; ++nf)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            sred[(wave * 2 + 0) * C + nf * 16 + 4 * kq + r] += ssum[nf * 4 + r];
            sred[(wave * 2 + 1) * C + nf * 16 + 4 * kq + r] += ssq[nf * 4 + r];
          }
      }
    }
    lgkm_wait0_h();
    halo_bar();        // every wave's patch reads of this tile retired
    halo_vm_wait16();  // this thread's next-patch loads landed; its 16 output stores may still fly
    store_patch(nxt);
    lgkm_wait0_h();
    halo_bar();        // the next patch is in LDS
  }
  if constexpr (STATS) {
    __syncthreads();
    if (tid < 2 * C) {
      const int k = tid / C, c = tid % C;
      float a = 0.f;
#pragma unroll
      for (int w = 0; w < STEM_WAVES; ++w) a += sred[(w * 2 + k) * C + c];
      P.stats[((long)blockIdx.x * 2 + k) * C + c] = a;
    }
  }
}

}  // namespace ca
