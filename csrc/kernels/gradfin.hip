// Batched gradient finalisation: the fixed-order reductions that turn per-block partials
// into parameter gradients -- split-K fp32 slabs -> weight gradient (splitk_reduce in
// gemm.hip) and column partials -> bias / LayerNorm gradients (col_finalize in rowops.hip)
// -- for up to FIN_MAX independent jobs in ONE launch.
//
// A BERT layer backward produces eight of them (four weight-gradient slab sets, the two
// LayerNorms' [dgamma | dbeta | dsum] partials, two bias column sums); each was its own
// 2-16 us launch.  The jobs travel by value in the kernel arguments (no descriptor upload,
// no extra copy dispatch); block b finds its job by a scan of the per-job block offsets.
// Every job keeps exactly the summation order of its standalone kernel, so results are
// bitwise those of the unbatched path.
#include "ca_common.h"

namespace {

constexpr int FIN_MAX = 8;

struct FinJob {
  int kind;           // 0: slabs src[S][n] -> out0 (fp32 / bf16) = sum + beta * out0
                      // 1: partials src[nparts][stride] -> out0 | out1 | out2 columns (N each)
  int nblocks;
  const float* src;
  int nparts;         // slabs S / partial rows
  int cb;             // kind 0: float4 columns per block
  long stride;        // kind 0: slab stride (= n) / kind 1: partial row stride
  long n;             // kind 0: elements / kind 1: N
  void* out0;
  float* out1;
  float* out2;
  int out_bf16;
  int accumulate;
  float beta;
};

struct FinArgs {
  FinJob j[FIN_MAX];
  int start[FIN_MAX + 1];
  int nj;
};

// large outputs (cb == 0): one float4 column per thread, slabs summed in order 0..S-1 with
// every load issued back to back -- bitwise gemm.hip splitk_reduce_cols_kernel
__device__ void fin_splitk_cols(const FinJob& J, int vb) {
  const long n4 = J.n / 4;
  const long v = (long)vb * 256 + threadIdx.x;
  if (v >= n4) return;
  const f4* p = reinterpret_cast<const f4*>(J.src) + v;
  f4 acc = p[0];
  int s = 1;
  for (; s + 4 <= J.nparts; s += 4) {
    const f4 a = p[(long)s * n4], b = p[(long)(s + 1) * n4], c = p[(long)(s + 2) * n4], d = p[(long)(s + 3) * n4];
    acc += a;
    acc += b;
    acc += c;
    acc += d;
  }
  for (; s < J.nparts; ++s) acc += p[(long)s * n4];
  if (J.out_bf16) {
    bf16_t* o = reinterpret_cast<bf16_t*>(J.out0) + v * 4;
    if (J.beta != 0.f) {
      const us4 old = *reinterpret_cast<const us4*>(o);
      for (int j = 0; j < 4; ++j) acc[j] += J.beta * bf2f(old[j]);
    }
    us4 r;
    for (int j = 0; j < 4; ++j) r[j] = f2bf(acc[j]);
    *reinterpret_cast<us4*>(o) = r;
  } else {
    float* o = reinterpret_cast<float*>(J.out0) + v * 4;
    if (J.beta != 0.f) acc += J.beta * *reinterpret_cast<const f4*>(o);
    *reinterpret_cast<f4*>(o) = acc;
  }
}

__device__ void fin_splitk(const FinJob& J, int vb, f4* red) {
  const long n4 = J.n / 4;
  const int CB = J.cb, SL = 256 / CB;
  const int col = threadIdx.x % CB, sl = threadIdx.x / CB;
  const long v = (long)vb * CB + col;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  if (v < n4) {
#pragma unroll 4
    for (int s = sl; s < J.nparts; s += SL) acc += *reinterpret_cast<const f4*>(J.src + (long)s * J.stride + v * 4);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = SL / 2; w > 0; w >>= 1) {
    if (sl < w) red[threadIdx.x] += red[threadIdx.x + w * CB];
    __syncthreads();
  }
  if (sl != 0 || v >= n4) return;
  acc = red[col];
  if (J.out_bf16) {
    bf16_t* o = reinterpret_cast<bf16_t*>(J.out0) + v * 4;
    if (J.beta != 0.f) {
      const us4 old = *reinterpret_cast<const us4*>(o);
      for (int j = 0; j < 4; ++j) acc[j] += J.beta * bf2f(old[j]);
    }
    us4 r;
    for (int j = 0; j < 4; ++j) r[j] = f2bf(acc[j]);
    *reinterpret_cast<us4*>(o) = r;
  } else {
    float* o = reinterpret_cast<float*>(J.out0) + v * 4;
    if (J.beta != 0.f) acc += J.beta * *reinterpret_cast<const f4*>(o);
    *reinterpret_cast<f4*>(o) = acc;
  }
}

__device__ void fin_cols(const FinJob& J, int vb, float (*red)[17]) {
  const int cl = threadIdx.x & 15, pl = threadIdx.x >> 4;
  const long N = J.n;
  const long c = (long)vb * 16 + cl;
  const long total = J.out2 ? 3 * N : (J.out1 ? 2 * N : N);
  float t = 0.f;
  if (c < total) {
#pragma unroll 4
    for (int p = pl; p < J.nparts; p += 16) t += J.src[(long)p * J.stride + c];
  }
  red[pl][cl] = t;
  __syncthreads();
  if (pl != 0 || c >= total) return;
  t = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) t += red[k][cl];
  const int k = (int)(c / N);
  float* dst = k == 0 ? reinterpret_cast<float*>(J.out0) : (k == 1 ? J.out1 : J.out2);
  if (!dst) return;
  float* o = dst + (c - k * N);
  *o = J.accumulate ? *o + t : t;
}

__global__ void __launch_bounds__(256) grad_fin_kernel(FinArgs a) {
  __shared__ __attribute__((aligned(16))) f4 red[256];
  const int b = blockIdx.x;
  int j = 0;
  while (j + 1 < a.nj && b >= a.start[j + 1]) ++j;
  const int vb = b - a.start[j];
  if (a.j[j].kind == 0 && a.j[j].cb == 0) fin_splitk_cols(a.j[j], vb);
  else if (a.j[j].kind == 0) fin_splitk(a.j[j], vb, red);
  else fin_cols(a.j[j], vb, reinterpret_cast<float(*)[17]>(red));
}

}  // namespace

extern "C" {

// jobs: n rows of 12 u64 fields {kind, src, nparts, stride, n, out0, out1, out2, out_bf16,
// accumulate, -, -} and betas[n]; launched in groups of FIN_MAX.
int ca_grad_finalize_multi(const uint64_t* jobs, const float* betas, int n, hipStream_t s) {
  for (int g0 = 0; g0 < n; g0 += FIN_MAX) {
    FinArgs a{};
    a.nj = n - g0 < FIN_MAX ? n - g0 : FIN_MAX;
    int blocks = 0;
    for (int i = 0; i < a.nj; ++i) {
      const uint64_t* r = jobs + (long)(g0 + i) * 12;
      FinJob& J = a.j[i];
      J.kind = (int)r[0];
      J.src = reinterpret_cast<const float*>(r[1]);
      J.nparts = (int)r[2];
      J.stride = (long)r[3];
      J.n = (long)r[4];
      J.out0 = reinterpret_cast<void*>(r[5]);
      J.out1 = reinterpret_cast<float*>(r[6]);
      J.out2 = reinterpret_cast<float*>(r[7]);
      J.out_bf16 = (int)r[8];
      J.accumulate = (int)r[9];
      J.beta = betas[g0 + i];
      if (J.kind == 0) {
        if (J.n % 4) return -3;
        const long n4 = J.n / 4;
        J.cb = n4 < 16L * 512 ? 4 : (n4 < 64L * 512 ? 16 : 0);  // as ca_splitk_reduce (0: column kernel)
        J.nblocks = J.cb ? (int)((n4 + J.cb - 1) / J.cb) : (int)((n4 + 255) / 256);
      } else if (J.kind == 1) {
        const long total = J.out2 ? 3 * J.n : (J.out1 ? 2 * J.n : J.n);
        J.nblocks = (int)((total + 15) / 16);
      } else {
        return -1;
      }
      a.start[i] = blocks;
      blocks += J.nblocks;
    }
    a.start[a.nj] = blocks;
    if (blocks > 0) {
      grad_fin_kernel<<<blocks, 256, 0, s>>>(a);
      CA_LAUNCH_CHECK();
    }
  }
  return 0;
}

}  // extern "C"
