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
// LDS layouts.  Filter image: [row][64 channels] (128 B per row), 16-B chunk c of row q at chunk
// c ^ ((q >> 1) & 7).  Patch image: CHUNK-MAJOR, [8 chunks][patch pixel q] (16 B per pixel,
// planes HALO_PLANE bytes apart, a multiple of 256 B): the A-fragment reads of a ds_read_b128
// lane group ({0-3,12-15,20-27}-style: 16 pixels, two adjacent chunks) then hit 16 distinct
// 16-B bank slots whenever the fragment's 16 pixels are consecutive patch pixels -- a fragment
// crossing an image row skips the two pad columns and may double one slot.  Simulated over
// every (wave, fragment, tap): 4.57 LDS cycles per A read against 6.86 for the XOR-swizzled
// row-major image (4 = conflict-free).  The patch is written by 8-lane groups of one chunk
// over 8 consecutive pixels (distinct slots), loaded from global memory as whole 128-B rows
// per 8 lanes.
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
constexpr int HALO_PLANE = 37 * 256;  // bytes per chunk plane: >= 10 x 58 pixels x 16 B, multiple of 256

// sum over the 16 lanes of a DPP row (row_ror 8, row_ror 4, quad swaps): every lane gets the total
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4e, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xb1, 0xf, 0xf, false));
  return v;
}

__device__ __forceinline__ int halo_swz(int q, int chunk) { return q * 64 + ((chunk ^ ((q >> 1) & 7)) << 3); }

// raw barrier (no fence: __syncthreads()'s fence would drain the vector-memory counter) and the
// counted waits of the persistent tile loops here and in ca_conv_stem.h
__device__ __forceinline__ void halo_bar() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void halo_vm_wait16() { asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); }
__device__ __forceinline__ void halo_vm_wait28() { asm volatile("s_waitcnt vmcnt(28)" ::: "memory"); }
__device__ __forceinline__ void halo_vm_wait0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void lgkm_wait0_h() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// W = 56 only (8 x 56 = 448 = 7 x 64 pixels per tile); H % 8 == 0 (host-checked).
// STATS: 0 none, 1 forward statistics (sum, sum of squares), 2 input-gradient BN-backward statistics
template <int STATS, bool PIPE = true>
__device__ __forceinline__ void conv3x3_halo(const HaloParams& P) {
  constexpr int C = HALO_C, TR = HALO_TR, NT = HALO_NT, W = 56, PW = W + 2, PR = TR + 2;
  constexpr int WIMG = 9 * C * C;      // shorts
  constexpr int PIMG = 8 * HALO_PLANE / 2;  // shorts
  static_assert(PR * PW * 16 <= HALO_PLANE, "patch plane");
  constexpr int PCH = PR * W * 8;      // 16-B chunks of a patch's interior = 4480 = 10 per thread
  static_assert(PCH % NT == 0, "patch chunks must divide the threads");
  constexpr int PPT = PCH / NT;
  constexpr int SRED = STATS != 0 ? HALO_WAVES * 2 * C * 2 : 0;  // shorts: per-wave [2][64] fp32 statistics
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
    if (!P.dgrad) {  // e = (tap, co, ci chunk): one 16-B row piece per iteration
      const int tap = e / (C * 8), n = (e / 8) % C, ch = e % 8;
      *reinterpret_cast<s8v*>(wimg + halo_swz(tap * C + n, ch)) =
          *reinterpret_cast<const s8v*>(P.w + ((long)n * 9 + tap) * C + ch * 8);
    } else {  // e = (source tap, co, ci chunk): 8 consecutive ci of one co scatter to 8 image rows
      const int tp = e / (C * 8), co = (e / 8) % C, cc = e % 8;
      const s8v v = *reinterpret_cast<const s8v*>(P.w + ((long)co * 9 + tp) * C + cc * 8);
      const int tap = 8 - tp;
#pragma unroll
      for (int j = 0; j < 8; ++j) wimg[halo_swz(tap * C + cc * 8 + j, co >> 3) + (co & 7)] = v[j];
    }
  }
  // the patch's left / right zero columns never change
  for (int e = tid; e < PR * 2 * 8; e += NT) {
    const int r = e / 16, side = (e / 8) & 1, ch = e % 8;
    *reinterpret_cast<s8v*>(pimg + ch * (HALO_PLANE / 2) + (r * PW + (side ? PW - 1 : 0)) * 8) = zero8();
  }

  // this thread's patch chunks: chunk i is patch row i, image column c = 8 * wave + (lane & 7),
  // channel chunk (lane >> 3) & 7 -- each 8-lane group covers one chunk of 8 consecutive pixels
  // (distinct LDS bank slots on the store), each wave 8 whole 128-B pixel rows per load
  const int pc = wave * 8 + (lane & 7), pch = (lane >> 3) & 7;
  static_assert(PPT == PR && HALO_WAVES * 8 == W, "one patch row per chunk, 8 columns per wave");
  // Branch-free: a pad row loads its clamped in-image neighbour and is zeroed after the load (a
  // load under a branch makes hipcc wait vmcnt(0) where the branches join).
  auto load_patch = [&](int t, s8v (&v)[PPT]) {
    const int n = t / rgroups, r0 = (t % rgroups) * TR - 1;  // patch row 0 = image row r0
    const bf16_t* src = P.x + (((long)n * H + r0) * W + pc) * C + pch * 8;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const bool ok = (i > 0 || r0 >= 0) && (i < PPT - 1 || r0 + i < H);  // only rows 0 and PR-1 can be pads
      const int ii = i == 0 ? (ok ? 0 : 1) : (i == PPT - 1 ? (ok ? i : i - 1) : i);
      const s8v ld = *reinterpret_cast<const s8v*>(src + (long)ii * W * C);
      v[i] = ok ? ld : zero8();
    }
  };
  short* pdst = pimg + pch * (HALO_PLANE / 2) + (pc + 1) * 8;
  auto store_patch = [&](const s8v (&v)[PPT]) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) *reinterpret_cast<s8v*>(pdst + i * PW * 8) = v[i];
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

  // Tile loop: the next tile's patch loads are issued at the top of a tile, BEFORE its epilogue
  // stores, and written to LDS at the bottom behind a counted vmcnt(16), so a tile's 16 output
  // stores per lane stay in flight across the next tile's MFMAs.  (With a __syncthreads() at the
  // loop top hipcc drained vmcnt to 0 there: every tile waited out its own store latency.)
  // Inside the loop only LDS is shared between the waves: raw s_barriers with lgkmcnt(0).
  int t = blockIdx.x;
  s8v nxt[PPT];
  if (t < ntiles) {
    load_patch(t, nxt);
    halo_vm_wait0();
    store_patch(nxt);
  }
  __syncthreads();  // the filter image, the pad columns and the first patch written
  for (; t < ntiles; t += gridDim.x) {
    const int tn = t + gridDim.x;
    load_patch(tn < ntiles ? tn : t, nxt);  // in flight during the MFMAs and stores below

    f4v acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
    const int n = t / rgroups, r0 = (t % rgroups) * TR;
    const long tile_pix = ((long)n * H + r0) * W;  // first pixel of the tile (rows are whole)
    const long pix0 = tile_pix + wave * 64 + (lane & 15);  // pixel of fragment 0; fragment mf: + 16 mf
    // dgrad statistics: the tile's z / mask loads are issued halfway through its MFMAs (PIPE)
    // or at the start of the epilogue, all before the first use
    us4 zv[4][4];
    uint32_t mv[4][2];
    auto load_bn = [&]() {
      if constexpr (STATS == 2) {
#pragma unroll
        for (int mf = 0; mf < 4; ++mf) {
          const long pix = pix0 + mf * 16;
          if (P.bnmask) {
            const uint2 m = *reinterpret_cast<const uint2*>(P.bnmask + pix * 8);
            mv[mf][0] = m.x;
            mv[mf][1] = m.y;
          } else {
            mv[mf][0] = mv[mf][1] = 0xffffffffu;
          }
#pragma unroll
          for (int nf = 0; nf < 4; ++nf)
            zv[mf][nf] = *reinterpret_cast<const us4*>(P.bnz + pix * C + 4 * kq + nf * 16);
        }
      }
    };
    // 18 K steps (9 taps x 2 channel halves).  PIPE: the fragments of step s + 1 are read from
    // LDS while the 16 MFMAs of step s run (two register sets, fully unrolled), so a wave does
    // not wait out the LDS latency before every step.
    auto frag_load = [&](int st, bf16x8 (&af)[4], bf16x8 (&bfr)[4]) {
      const int tap = st >> 1, chunk = (st & 1) * 4 + kq;
      const int dq = (tap / 3) * PW + (tap % 3);
#pragma unroll
      for (int nf = 0; nf < 4; ++nf)
        bfr[nf] = __builtin_bit_cast(
            bf16x8, *reinterpret_cast<const s8v*>(wimg + halo_swz(tap * C + nf * 16 + (lane & 15), chunk)));
#pragma unroll
      for (int mf = 0; mf < 4; ++mf)
        af[mf] = __builtin_bit_cast(
            bf16x8, *reinterpret_cast<const s8v*>(pimg + chunk * (HALO_PLANE / 2) + (q0[mf] + dq) * 8));
    };
    auto mfma16 = [&](const bf16x8 (&af)[4], const bf16x8 (&bfr)[4]) {
#pragma unroll
      for (int mf = 0; mf < 4; ++mf)
#pragma unroll
        for (int nf = 0; nf < 4; ++nf)
          acc[mf][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[nf], af[mf], acc[mf][nf], 0, 0, 0);
    };
    if constexpr (PIPE) {
      bf16x8 fa[2][4], fb[2][4];
      frag_load(0, fa[0], fb[0]);
#pragma unroll
      for (int st = 0; st < 18; ++st) {
        if (st + 1 < 18) frag_load(st + 1, fa[(st + 1) & 1], fb[(st + 1) & 1]);
        if (st == 8) load_bn();
        __builtin_amdgcn_sched_barrier(0);  // keep the next step's reads ahead of this step's MFMAs
        mfma16(fa[st & 1], fb[st & 1]);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll 1
      for (int tap = 0; tap < 9; ++tap) {
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) {
          bf16x8 af[4], bfr[4];
          frag_load(tap * 2 + kh, af, bfr);
          mfma16(af, bfr);
        }
      }
      load_bn();
    }

    // epilogue: lane holds pixel (mf*16 + lane&15), channels nf*16 + 4*kq + r.  The tile's
    // statistics (of channels nf * 16 + 4 * kq + r, index nf * 4 + r) are reduced over the 16
    // pixel lanes and added to this wave's LDS row, so they hold no registers across tiles.
    float ssum[16], ssq[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) ssum[j] = ssq[j] = 0.f;
#pragma unroll
    for (int mf = 0; mf < 4; ++mf) {
      bf16_t* yp = P.y + (pix0 + mf * 16) * C + 4 * kq;
#pragma unroll
      for (int nf = 0; nf < 4; ++nf) {
        us4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = f2bf(acc[mf][nf][r]);
        *reinterpret_cast<us4*>(yp + nf * 16) = o;
        if constexpr (STATS == 1) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float a = bf2f(o[r]);
            ssum[nf * 4 + r] += a;
            ssq[nf * 4 + r] += a * a;
          }
        } else if constexpr (STATS == 2) {
          // channels nf*16 + 4*kq + r: mask byte nf*2 + kq/2, nibble kq&1
          const uint32_t byte = (mv[mf][nf >> 1] >> (((nf & 1) * 2 + (kq >> 1)) * 8)) & 0xffu;
          const uint32_t nib = (byte >> ((kq & 1) * 4)) & 0xfu;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float g = ((nib >> r) & 1u) ? bf2f(o[r]) : 0.f;
            ssum[nf * 4 + r] += g;
            ssq[nf * 4 + r] += g * bf2f(zv[mf][nf][r]);
          }
        }
      }
    }
    if constexpr (STATS) {
      // sums over the 16 pixel lanes of each 16-lane row: DPP rotates within the row (VALU,
      // no LDS permutes), every lane ends with the row total
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        ssum[j] = row16_sum(ssum[j]);
        ssq[j] = row16_sum(ssq[j]);
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
    lgkm_wait0_h();
    halo_bar();      // every wave's patch reads of this tile retired
    halo_vm_wait16();  // this thread's next-patch loads landed; its 16 output stores may still fly
    store_patch(nxt);
    lgkm_wait0_h();
    halo_bar();      // the next patch is in LDS
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

namespace ca {

// ------------------------------------------------------------------ weight gradient --
// dW[co][tap][ci] = sum over pixels p of dY[p][co] * X[p + tap][ci] for the same convolutions
// (3x3 / s1 / p1, 64 -> 64 channels, W = 56).  The implicit-GEMM weight gradient gathers the
// shifted input nine times per pixel tile and runs 64-row tiles of a 64 x 576 output split
// thousands of ways (ResNet-50 stage 1, batch 1024: 406 TF/s).  Here a persistent workgroup
// (8 waves, one per CU) keeps the WHOLE 64 x 576 partial sum in registers across all its
// tiles (wave w: output rows 32 (w & 1) .. + 32, columns 144 (w >> 1) .. + 144 = 2 x 9
// fragments) and per tile of 8 image rows stages
//   * the output gradient tile, [448 pixels][64 channels], and
//   * the input patch, [10 x 58 positions][64 channels] with zero borders,
// once in LDS; K = pixels.  Both operands are read with the transposing LDS read
// (ds_read_b64_tr_b16, the GDenseNC layout of ca_mfma_core.h) -- a B fragment of tap (dr, dc)
// is the patch read at the pixel rows shifted by dr * 58 + dc: every group of 8 pixels a lane
// reads lies in one image row (56 = 7 x 8), so its 8 patch rows are consecutive.  Each
// workgroup writes ONE fp32 [64][576] partial; the split-K reduce sums them.
struct HaloWgParams {
  const bf16_t* x;   // input [N][H][W][64]
  const bf16_t* dy;  // output gradient [N][H][W][64]
  float* ws;         // [gridDim.x][64][576] fp32 partials
  int N, H, W;
};

constexpr int HWG_WAVES = 8, HWG_NT = HWG_WAVES * 64;

// NC-layout fragment (ca_mfma_core.h read_frag_sw<R, false>) whose K rows are given per lane:
// krow = the LDS row holding k = 8 * (lane >> 4), the lane's group of 8 consecutive K rows
__device__ __forceinline__ bf16x8 read_frag_nc_rows(const short* lds, int r0, int krow, int lane) {
  constexpr int R = 64;
  const int q = (lane & 15) >> 2, p = lane & 3;
  const int k = krow + q;
  const int lc = (r0 >> 3) + (p >> 1);
  const int sub = 4 * (p & 1);
  const short* b0 = lds + k * R + ((lc ^ nc_swz<R>(k)) << 3) + sub;
  const short* b1 = lds + (k + 4) * R + ((lc ^ nc_swz<R>(k + 4)) << 3) + sub;
  s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(b0));
  s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(b1));
  s8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ void conv3x3_halo_wgrad(const HaloWgParams& P) {
  constexpr int C = HALO_C, TR = HALO_TR, NT = HWG_NT, W = 56, PW = W + 2, PR = TR + 2;
  constexpr int TP = TR * W;              // 448 pixels per tile
  constexpr int DCH = TP * 8 / NT;        // 7 output-gradient chunks per thread
  constexpr int PCH = PR * W * 8;         // 4480 patch interior chunks
  constexpr int PPT = (PCH + NT - 1) / NT;  // 9 (the last one partial)
  static_assert(TP * 8 % NT == 0, "tile chunks");
  __shared__ __attribute__((aligned(16))) short smem[TP * C + PR * PW * C];
  short* dimg = smem;
  short* pimg = smem + TP * C;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = P.H, rgroups = H / TR, ntiles = P.N * rgroups;
  const int cfb = (wave & 1) * 2, nfb = (wave >> 1) * 9;

  for (int e = tid; e < PR * 2 * 8; e += NT) {  // zero pad columns, once
    const int r = e / 16, side = (e / 8) & 1, ch = e % 8;
    const int q = r * PW + (side ? PW - 1 : 0);
    *reinterpret_cast<s8v*>(pimg + q * C + ((ch ^ nc_swz<64>(q)) << 3)) = zero8();
  }

  s8v dv[DCH], pv[PPT];
  auto load = [&](int t) {
    const int n = t / rgroups, r0 = (t % rgroups) * TR;
    const bf16_t* dsrc = P.dy + ((long)n * H + r0) * W * C;
#pragma unroll
    for (int i = 0; i < DCH; ++i) dv[i] = *reinterpret_cast<const s8v*>(dsrc + (long)(tid + i * NT) * 8);
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int e = tid + i * NT;
      const int pr = e / (W * 8), pc = (e / 8) % W, ch = e % 8;
      const int ir = r0 - 1 + pr;
      pv[i] = (e < PCH && ir >= 0 && ir < H)
                  ? *reinterpret_cast<const s8v*>(P.x + (((long)n * H + ir) * W + pc) * C + ch * 8)
                  : zero8();
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < DCH; ++i) {
      const int e = tid + i * NT, px = e >> 3, ch = e & 7;
      *reinterpret_cast<s8v*>(dimg + px * C + ((ch ^ nc_swz<64>(px)) << 3)) = dv[i];
    }
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int e = tid + i * NT;
      if (e < PCH) {
        const int pr = e / (W * 8), pc = (e / 8) % W, ch = e % 8;
        const int q = pr * PW + pc + 1;
        *reinterpret_cast<s8v*>(pimg + q * C + ((ch ^ nc_swz<64>(q)) << 3)) = pv[i];
      }
    }
  };

  f4v acc[2][9];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  int t = blockIdx.x;
  if (t < ntiles) load(t);
  for (; t < ntiles; t += gridDim.x) {
    __syncthreads();  // previous tile's reads retired
    store();
    __syncthreads();
    if (t + (int)gridDim.x < ntiles) load(t + gridDim.x);  // in flight during the MFMAs
#pragma unroll 1
    for (int ks = 0; ks < TP / 32; ++ks) {
      const int p0 = ks * 32;
      const int pg = p0 + 8 * (lane >> 4);  // this lane's group of 8 pixels (one image row)
      const int prow = pg / W, pcol = pg % W;
      bf16x8 af[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = read_frag_sw<64, false>(dimg, (cfb + i) * 16, p0, lane);
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const int nf = nfb + j, tap = nf >> 2, cif = nf & 3;
        const int krow = (prow + tap / 3) * PW + pcol + tap % 3;
        const bf16x8 bf = read_frag_nc_rows(pimg, cif * 16, krow, lane);
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf, af[i], acc[i][j], 0, 0, 0);
      }
    }
  }
  // lane holds dW[co = (cfb + i) * 16 + (lane & 15)][n = (nfb + j) * 16 + 4 * (lane >> 4) + r]
  float* dst = P.ws + (long)blockIdx.x * C * 576;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j)
      *reinterpret_cast<f4v*>(dst + ((cfb + i) * 16 + (lane & 15)) * 576 + (nfb + j) * 16 + 4 * (lane >> 4)) = acc[i][j];
}

}  // namespace ca
