// Standalone GEMM core benchmark + numerics check (no Python, no torch): the fast
// edit -> measure loop for the MFMA cores in csrc/include.  Every variant is timed in the
// same process on the same random operands (uniform [-1, 1), cdna_hip_programming.md
// §5.4 rules 24/25) and checked against an fp32 reference GEMM computed on the GPU.
//
//   build:  python -m cloud_amd._build gemm_bench      (-> bin/gemm_bench)
//   run:    bin/gemm_bench [iters] M,N,K,layout ...   layout 0 = NT (fwd), 1 = NN (dgrad), 2 = TN (wgrad)
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "ca_gemm256.h"
#include "ca_gemm256p8.h"
#include "ca_gemm_w4.h"

using namespace ca;

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

__global__ void init_uniform(bf16_t* p, long n, uint32_t seed) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (long)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    const float u = (float)(x >> 8) * (1.0f / 16777216.0f) * 2.f - 1.f;
    p[i] = f2bf(u);
  }
}

// reference: C[m][n] = sum_k A(m,k) B(k,n) in fp32, rows m = r * row_step + r % row_step only
// (every residue of the row index within a 16-row MFMA fragment is sampled)
__global__ void ref_gemm(const bf16_t* A, long lda, const bf16_t* B, long ldb, int layout, float* C, int M, int N, int K,
                         int row_step, int rows) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const int r = blockIdx.y;
  if (n >= N || r >= rows) return;
  int m = r * row_step + r % row_step;
  if (m >= M) m = M - 1;
  float s = 0.f;
  for (int k = 0; k < K; ++k) {
    const float a = layout == 2 ? bf2f(A[(long)k * lda + m]) : bf2f(A[(long)m * lda + k]);
    const float b = layout == 0 ? bf2f(B[(long)n * ldb + k]) : bf2f(B[(long)k * ldb + n]);
    s += a * b;
  }
  C[(long)r * N + n] = s;
}

template <template <int, int, int> class GA, template <int, int, int> class GB, bool ST>
__global__ void __launch_bounds__(512) k256(CoreParams P) {
  mfma_gemm_256<GA, GB, EPI_BF16, ST>(P);
}

template <template <int, int, int> class GA, template <int, int, int> class GB, int PHASES>
__global__ void __launch_bounds__(512) kp8(CoreParams P) {
  mfma_gemm_256p8<GA, GB, EPI_BF16, PHASES>(P);
}

template <template <int, int, int> class GA, template <int, int, int> class GB>
__global__ void __launch_bounds__(512) kp8sk(CoreParams P, SkParams S) {
  mfma_gemm_256p8_sk<GA, GB, EPI_BF16>(P, S);
}

template <template <int, int, int> class GA, template <int, int, int> class GB>
__global__ void __launch_bounds__(512) k256x128(CoreParams P) {
  mfma_gemm_256x128<GA, GB, EPI_BF16>(P);
}

template <template <int, int, int> class GA, template <int, int, int> class GB>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) k128(CoreParams P) {
  mfma_gemm_glds<128, 128, 2, 2, GA, GB, EPI_BF16>(P);
}

// 96-column tiles for BERT's N = 768 shapes at M = 8192 (forward NT only: the N-contiguous
// loaders need R / 8 to divide the thread count): 128 x 96 -> 512 tiles = 2 per CU exactly,
// 256 x 96 -> 256 tiles = 1 per CU (the 128 x 128 core's 384 tiles leave half the CUs a second
// round)
template <template <int, int, int> class GA, template <int, int, int> class GB>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) k128x96(CoreParams P) {
  mfma_gemm_glds<128, 96, 2, 2, GA, GB, EPI_BF16>(P);
}
template <template <int, int, int> class GA, template <int, int, int> class GB>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) k256x96(CoreParams P) {
  mfma_gemm_glds<256, 96, 2, 2, GA, GB, EPI_BF16>(P);
}
// the 128 x 64 tile the dispatcher runs for BERT's N = 768 forwards (768 tiles = 3 rounds)
template <template <int, int, int> class GA, template <int, int, int> class GB>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) k128x64(CoreParams P) {
  mfma_gemm_glds<128, 64, 2, 2, GA, GB, EPI_BF16>(P);
}
static void launch128x64(const CoreParams& p, int layout, dim3 g, hipStream_t s) {
  if (layout == 0) k128x64<GDenseKC, GDenseKC><<<g, 256, 0, s>>>(p);
  else if (layout == 1) k128x64<GDenseKC, GDenseNC><<<g, 256, 0, s>>>(p);
  else k128x64<GDenseNC, GDenseNC><<<g, 256, 0, s>>>(p);
}
// the same tile with the DMA of K tile t+1 in flight during tile t (two LDS stages, 48 KB:
// three blocks per CU still fit -- the shape only has three per CU), 4 or 8 waves
template <template <int, int, int> class GA, template <int, int, int> class GB>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) k128x64s2(CoreParams P) {
  mfma_gemm_glds<128, 64, 2, 2, GA, GB, EPI_BF16, 2>(P);
}
template <template <int, int, int> class GA, template <int, int, int> class GB>
__global__ void __launch_bounds__(512) k128x64w8(CoreParams P) {
  mfma_gemm_glds<128, 64, 4, 2, GA, GB, EPI_BF16, 2>(P);
}
static void launch128x64s2(const CoreParams& p, int layout, dim3 g, hipStream_t s) {
  if (layout == 0) k128x64s2<GDenseKC, GDenseKC><<<g, 256, 0, s>>>(p);
  else if (layout == 1) k128x64s2<GDenseKC, GDenseNC><<<g, 256, 0, s>>>(p);
  else k128x64s2<GDenseNC, GDenseNC><<<g, 256, 0, s>>>(p);
}
static void launch128x64w8(const CoreParams& p, int layout, dim3 g, hipStream_t s) {
  if (layout == 0) k128x64w8<GDenseKC, GDenseKC><<<g, 512, 0, s>>>(p);
  else if (layout == 1) k128x64w8<GDenseKC, GDenseNC><<<g, 512, 0, s>>>(p);
  else k128x64w8<GDenseNC, GDenseNC><<<g, 512, 0, s>>>(p);
}
static void launch128x96(const CoreParams& p, int layout, dim3 g, hipStream_t s) {
  if (layout == 0) k128x96<GDenseKC, GDenseKC><<<g, 256, 0, s>>>(p);
}
static void launch256x96(const CoreParams& p, int layout, dim3 g, hipStream_t s) {
  if (layout == 0) k256x96<GDenseKC, GDenseKC><<<g, 256, 0, s>>>(p);
}

// four waves, one workgroup per CU, accumulators in AGPRs (ca_gemm_w4.h)
template <int BN, template <int, int, int> class GA, template <int, int, int> class GB, int DIAG = 0>
__global__ void __launch_bounds__(256, 1) kw4(CoreParams P) {
  mfma_gemm_w4<BN, GA, GB, EPI_BF16, DIAG>(P);
}
template <int BN, int DIAG = 0>
static void launchw4(const CoreParams& p, int layout, dim3 g, hipStream_t s) {
  if (layout == 0) kw4<BN, GDenseKC, GDenseKC, DIAG><<<g, 256, 0, s>>>(p);
  else if (layout == 1 && DIAG == 0) kw4<BN, GDenseKC, GDenseNC><<<g, 256, 0, s>>>(p);
}

struct Variant {
  const char* name;
  int bm, bn;
  void (*launch)(const CoreParams&, int layout, dim3 grid, hipStream_t);
};

template <bool ST>
static void launch256_t(const CoreParams& p, int layout, dim3 g, hipStream_t s) {
  if (layout == 0) k256<GDenseKC32, GDenseKC32, ST><<<g, 512, 0, s>>>(p);
  else if (layout == 1) k256<GDenseKC32, GDenseNC, ST><<<g, 512, 0, s>>>(p);
  else k256<GDenseNC, GDenseNC, ST><<<g, 512, 0, s>>>(p);
}
static void launch256(const CoreParams& p, int layout, dim3 g, hipStream_t s) { launch256_t<false>(p, layout, g, s); }

template <int PHASES>
static void launchp8(const CoreParams& p, int layout, dim3 g, hipStream_t s) {
  if (layout == 0) kp8<GDenseKC, GDenseKC, PHASES><<<g, 512, 0, s>>>(p);
  else if (layout == 1) kp8<GDenseKC, GDenseNC, PHASES><<<g, 512, 0, s>>>(p);
  else kp8<GDenseNC, GDenseNC, PHASES><<<g, 512, 0, s>>>(p);
}

// stream-K: one workgroup per CU over all (tile, K iteration) pairs; the grid argument is
// ignored (the 256 x 256 tile count comes from p)
static void launchp8sk(const CoreParams& p, int layout, dim3, hipStream_t s) {
  static float* part = nullptr;
  static int* ticket = nullptr;
  int dev = 0, cus = 256;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  if (!part) {
    CHECK(hipMalloc(&part, (size_t)cus * 256 * 256 * 4));
    CHECK(hipMalloc(&ticket, 65536 * 4));
    CHECK(hipMemset(ticket, 0, 65536 * 4));
  }
  SkParams S{};
  const int tiles = ((p.M + 255) / 256) * ((p.N + 255) / 256);
  S.part = part;
  S.ticket = ticket;
  S.err_index = 65535;
  S.ipt = (p.K + 63) / 64;
  S.total = tiles * S.ipt;
  const int g = (int)(S.total < cus ? S.total : cus);
  if (layout == 0) kp8sk<GDenseKC, GDenseKC><<<g, 512, 0, s>>>(p, S);
  else if (layout == 1) kp8sk<GDenseKC, GDenseNC><<<g, 512, 0, s>>>(p, S);
  else kp8sk<GDenseNC, GDenseNC><<<g, 512, 0, s>>>(p, S);
}

static void launch256x128(const CoreParams& p, int layout, dim3 g, hipStream_t s) {
  if (layout == 0) k256x128<GDenseKC, GDenseKC><<<g, 512, 0, s>>>(p);
  else if (layout == 1) k256x128<GDenseKC, GDenseNC><<<g, 512, 0, s>>>(p);
  else k256x128<GDenseNC, GDenseNC><<<g, 512, 0, s>>>(p);
}

// (a 128 x 192 variant of the glds core was measured in round 5, profiles/r5_s6/r5s6_gb.log:
// 15-40 % slower than 128 x 128 on every BERT shape and wrong -- the core's epilogue layout
// assumes a power-of-two BN -- and was removed)

static void launch128(const CoreParams& p, int layout, dim3 g, hipStream_t s) {
  if (layout == 0) k128<GDenseKC, GDenseKC><<<g, 256, 0, s>>>(p);
  else if (layout == 1) k128<GDenseKC, GDenseNC><<<g, 256, 0, s>>>(p);
  else k128<GDenseNC, GDenseNC><<<g, 256, 0, s>>>(p);
}

// per-phase shader-cycle medians of the 256 core (GB_STAMP=1): R work, R -> barrier wait,
// M work, per wave group, for the K tile in the middle of each block's loop
static void stamp_report(const CoreParams& p0, int layout, dim3 g, hipStream_t s) {
  CoreParams p = p0;
  const long n = (long)g.x * 8 * 17;
  CHECK(hipMalloc(&p.stamps, n * 8));
  CHECK(hipMemsetAsync(p.stamps, 0, n * 8, s));
  for (int w = 0; w < 3; ++w) launch256_t<true>(p, layout, g, s);
  CHECK(hipStreamSynchronize(s));
  std::vector<unsigned long long> h(n);
  CHECK(hipMemcpy(h.data(), p.stamps, n * 8, hipMemcpyDeviceToHost));
  CHECK(hipFree(p.stamps));
  for (int grp = 0; grp < 2; ++grp) {
    std::vector<long> r, w, m;
    for (unsigned b = 0; b < g.x; ++b)
      for (int wv = grp * 4; wv < grp * 4 + 4; ++wv) {
        const unsigned long long* st = h.data() + ((long)b * 8 + wv) * 17;
        r.push_back((long)(st[1] - st[0]));
        w.push_back((long)(st[2] - st[1]));
        m.push_back((long)(st[3] - st[2]));
      }
    std::sort(r.begin(), r.end());
    std::sort(w.begin(), w.end());
    std::sort(m.begin(), m.end());
    printf("{\"stamps_group\": %d, \"R\": %ld, \"R_wait\": %ld, \"M\": %ld}\n", grp, r[r.size() / 2],
           w[w.size() / 2], m[m.size() / 2]);
  }
}

int main(int argc, char** argv) {
  int iters = 20;
  int a0 = 1;
  if (argc > 1 && !strchr(argv[1], ',')) {
    iters = atoi(argv[1]);
    a0 = 2;
  }
  std::vector<int> shapes;
  for (int a = a0; a < argc; ++a) {
    int M, N, K, L;
    if (sscanf(argv[a], "%d,%d,%d,%d", &M, &N, &K, &L) == 4) shapes.insert(shapes.end(), {M, N, K, L});
  }
  if (shapes.empty()) shapes = {4096, 4096, 4096, 0};
  const char* only = getenv("GB_VARIANTS");  // comma list of full variant names, e.g. "v256,glds128"
  Variant vars[] = {{"v256", 256, 256, launch256},
                    {"p8q4", 256, 256, launchp8<4>},
                    {"p8h2", 256, 256, launchp8<2>},
                    {"p8sk", 256, 256, launchp8sk},
                    {"w256x128", 256, 128, launch256x128},
                    {"glds128", 128, 128, launch128},
                    {"g128x64", 128, 64, launch128x64},
                    {"g128x64s2", 128, 64, launch128x64s2},
                    {"g128x64w8", 128, 64, launch128x64w8},
                    {"g128x96", 128, 96, launch128x96},
                    {"g256x96", 256, 96, launch256x96},
                    {"w4n256", 256, 256, launchw4<256>},
                    {"w4n192", 256, 192, launchw4<192>},
                    {"w4n160", 256, 160, launchw4<160>},
                    {"w4n128", 256, 128, launchw4<128>},
                    {"w4d1n256", 256, 256, launchw4<256, 1>},
                    {"w4d2n256", 256, 256, launchw4<256, 2>}};
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (size_t si = 0; si < shapes.size(); si += 4) {
    const int M = shapes[si], N = shapes[si + 1], K = shapes[si + 2], L = shapes[si + 3];
    bf16_t *A, *B, *C;
    const long na = (long)M * K, nb = (long)N * K, nc = (long)M * N;
    CHECK(hipMalloc(&A, na * 2));
    CHECK(hipMalloc(&B, nb * 2));
    CHECK(hipMalloc(&C, nc * 2));
    init_uniform<<<2048, 256, 0, s>>>(A, na, 0x1234u);
    init_uniform<<<2048, 256, 0, s>>>(B, nb, 0x9876u);
    const long lda = L == 2 ? M : K;  // TN: A stored [K][M]
    const long ldb = L == 0 ? K : N;  // NT: B [N][K]; NN/TN: B [K][N]
    const int row_step = M > 512 ? M / 509 : 1;
    const int rows = (M + row_step - 1) / row_step;
    float* R;
    CHECK(hipMalloc(&R, (long)rows * N * 4));
    ref_gemm<<<dim3((N + 255) / 256, rows), 256, 0, s>>>(A, lda, B, ldb, L, R, M, N, K, row_step, rows);
    std::vector<float> ref((long)rows * N);
    CHECK(hipMemcpyAsync(ref.data(), R, ref.size() * 4, hipMemcpyDeviceToHost, s));
    CHECK(hipStreamSynchronize(s));
    for (const Variant& v : vars) {
      if (only && !strstr(only, v.name)) continue;
      if ((v.launch == launch128x96 || v.launch == launch256x96) && L != 0) continue;
      if (strncmp(v.name, "w4", 2) == 0 && (L == 2 || (L == 1 && v.bn != 256 && v.bn != 128))) continue;
      CoreParams p{};
      p.A = A; p.lda = lda; p.B = B; p.ldb = ldb; p.C = C; p.ldc = N;
      p.M = M; p.N = N; p.K = K; p.k_per_split = K; p.split_xcd = 1;
      const int tiles = ((M + v.bm - 1) / v.bm) * ((N + v.bn - 1) / v.bn);
      const dim3 g(tiles, 1, 1);
      CHECK(hipMemsetAsync(C, 0xff, nc * 2, s));
      v.launch(p, L, g, s);
      CHECK(hipGetLastError());
      CHECK(hipStreamSynchronize(s));
      std::vector<bf16_t> out((long)rows * N);
      for (int r = 0; r < rows; ++r)
        CHECK(hipMemcpy(out.data() + (long)r * N, C + std::min((long)r * row_step + r % row_step, (long)M - 1) * N, (long)N * 2, hipMemcpyDeviceToHost));
      double num = 0, den = 0, maxe = 0;
      long bad = 0;
      for (long i = 0; i < (long)rows * N; ++i) {
        uint32_t ob = ((uint32_t)out[i]) << 16;
        float of;
        memcpy(&of, &ob, 4);
        const double o = of, r = ref[i];
        const double d = o - r;
        num += d * d;
        den += r * r;
        const double e = fabs(d) / (1.0 + fabs(r));
        if (!(e <= 0.05)) ++bad;
        if (e > maxe || e != e) maxe = e;
      }
      for (int w = 0; w < 3; ++w) v.launch(p, L, g, s);
      CHECK(hipEventRecord(e0, s));
      for (int it = 0; it < iters; ++it) v.launch(p, L, g, s);
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      ms /= iters;
      printf("{\"variant\": \"%s\", \"M\": %d, \"N\": %d, \"K\": %d, \"layout\": %d, \"us\": %.1f, \"TF\": %.1f, "
             "\"rel_l2\": %.3e, \"max_err\": %.3e, \"bad\": %ld}\n",
             v.name, M, N, K, L, ms * 1e3, 2.0 * M * N * K / ms / 1e9, sqrt(num / (den + 1e-30)), maxe, bad);
      fflush(stdout);
      if (getenv("GB_STAMP") && v.launch == launch256) stamp_report(p, L, g, s);
    }
    CHECK(hipFree(A));
    CHECK(hipFree(B));
    CHECK(hipFree(C));
    CHECK(hipFree(R));
  }
  return 0;
}
