// pybind11 face of the gfx950 kernels.  Every entry point takes raw device
// pointers (uintptr_t from torch.Tensor.data_ptr()) and the HIP stream handle
// (torch.cuda.current_stream().cuda_stream); shape/dtype validation happens in
// the Python layer (cloud_amd/ops/*).  A non-zero HIP status raises.
#include <atomic>
#include <mutex>
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <stdint.h>

#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;
typedef uint16_t bf16_t;

extern "C" {
int ca_sgd_step(float*, void*, int, float*, bf16_t*, const float*, const float*, long, int, int, hipStream_t);
int ca_adam_step(float*, void*, int, float*, float*, bf16_t*, const float*, const float*, long, int, int, hipStream_t);
int ca_rmsprop_step(float*, void*, int, float*, float*, bf16_t*, const float*, const float*, long, int, hipStream_t);
int ca_sumsq(const void*, int, long, float*, hipStream_t);
int ca_scale(void*, int, long, const float*, hipStream_t);
long ca_bn_workspace_floats(long, int);
int ca_bn_fwd(const bf16_t*, const bf16_t*, bf16_t*, long, int, const float*, const float*, float, float,
              float*, float*, float*, float*, float*, float*, int, uint8_t*, hipStream_t);
int ca_bn_apply(const bf16_t*, const bf16_t*, bf16_t*, long, int, const float*, int, hipStream_t);
int ca_bn_fwd_partials(const bf16_t*, const bf16_t*, bf16_t*, long, int, const float*, int, const float*, const float*,
                       float, float, float*, float*, float*, float*, float*, int, uint8_t*, float*, hipStream_t);
int ca_bn_bwd(const bf16_t*, const bf16_t*, const uint8_t*, const bf16_t*, long, int, const float*, const float*,
              const float*, bf16_t*, bf16_t*, float*, float*, float*, float*, int, hipStream_t);
int ca_bn_bwd_partials(const bf16_t*, const bf16_t*, const uint8_t*, const bf16_t*, long, int, const float*, int,
                       const float*, const float*, const float*, bf16_t*, bf16_t*, float*, float*, float*, float*, int,
                       hipStream_t);
int ca_gemm_bf16_bnstats(int, const bf16_t*, long, const bf16_t*, long, bf16_t*, long, int, int, int, float,
                         const bf16_t*, const uint8_t*, float*, hipStream_t);
long ca_conv_dgrad_stat_tiles(int, int, int, int, int);
long ca_conv_dgrad_stat_rows(int, int, int, int, int, int, int, int, int, int, int, float);
long ca_conv_stat_rows(int, int, int, int, int, int, int, int, int, int, int);
int ca_conv_wgrad_splits(int, int, int, int, int, int, int, int, int, int, int, int);
int ca_bn_fwd_partials_ex(const bf16_t*, const bf16_t*, const float*, bf16_t*, long, int, const float*, int,
                          const float*, const float*, float, float, float*, float*, float*, float*, float*, int,
                          uint8_t*, float*, hipStream_t);
int ca_gemm_xa(int, int, const bf16_t*, const bf16_t*, const uint8_t*, const float*, const float*, const float*,
               const float*, bf16_t*, uint8_t*, long, const bf16_t*, long, bf16_t*, long, int, int, int, float, const bf16_t*,
               const uint8_t*, const bf16_t*, const uint8_t*, float*, const bf16_t*, float*, hipStream_t);
int ca_gemm_xa_bwd_strided(const bf16_t*, const bf16_t*, const uint8_t*, const float*, const float*, const float*,
                           bf16_t*, long, const bf16_t*, long, bf16_t*, long, int, int, int, int, int, int, int,
                           hipStream_t);
int ca_gemm_xa_dw(const bf16_t*, const bf16_t*, const uint8_t*, const float*, const float*, const float*, long,
                  const bf16_t*, long, bf16_t*, long, int, int, int, float, const bf16_t*, const uint8_t*,
                  const bf16_t*, const uint8_t*, float*, const bf16_t*, float*, const bf16_t*, long, void*, int, float,
                  float*, int, hipStream_t);
int ca_dgrad_gemm(int, const bf16_t*, long, const bf16_t*, long, bf16_t*, long, int, int, int, float, const bf16_t*,
                  const uint8_t*, const bf16_t*, const uint8_t*, float*, hipStream_t, const bf16_t*, float*, int, int,
                  int);
int ca_conv_dgrad_bnstats(const bf16_t*, const bf16_t*, bf16_t*, int, int, int, int, int, int, int, int, int, int,
                          int, float, const bf16_t*, const uint8_t*, float*, hipStream_t);
int ca_u8_normalize(const uint8_t*, bf16_t*, long, int, const float*, const float*, hipStream_t);
int ca_stem_s2d(const bf16_t*, bf16_t*, int, int, int, int, int, int, int, hipStream_t);
int ca_softmax_xent(const void*, int, const int64_t*, int, int, float, float, float*, float*, void*, hipStream_t);
int ca_softmax_xent_batch(const void*, long, int, const int64_t*, int, int, float, float, float*, float*, void*, float*,
                          float,
                          hipStream_t);
int ca_maxpool_fwd(const bf16_t*, bf16_t*, uint8_t*, int, int, int, int, int, int, int, int, int, hipStream_t);
int ca_maxpool_bwd(const bf16_t*, const uint8_t*, bf16_t*, int, int, int, int, int, int, int, int, int, hipStream_t);
int ca_gap_fwd(const bf16_t*, void*, int, int, int, int, hipStream_t);
int ca_gap_bwd(const void*, int, bf16_t*, int, int, int, hipStream_t);
int ca_gmp_fwd(const bf16_t*, bf16_t*, float*, int, int, int, hipStream_t);
int ca_gmp_bwd(const void*, int, const bf16_t*, const bf16_t*, const float*, bf16_t*, int, int, int, hipStream_t);
int ca_gemm_bf16(int, const bf16_t*, long, const bf16_t*, long, bf16_t*, long, int, int, int, float*, float,
                 hipStream_t);
int ca_gemm_set_core(int);
int ca_gemm_set_xa_n256(int);
int ca_gemm_set_streamk(int);
int ca_gemm_experimental_built();
int ca_gemm_stat_rows(int, int, int, long, long, long);
int ca_bn_relu_maxpool_s2k3(const bf16_t*, const float*, bf16_t*, uint8_t*, int, int, int, int, int, int, hipStream_t);
int ca_maxpool_bnstats_parts(int, int, int, int);
int ca_maxpool_bwd_s2k3_bnstats(const bf16_t*, const bf16_t*, const uint8_t*, const bf16_t*, bf16_t*, float*, int, int,
                                int, int, int, int, hipStream_t);
int ca_maxpool_bwd_s2k3_bnapply(const bf16_t*, const bf16_t*, const uint8_t*, const bf16_t*, const float*, bf16_t*, int,
                                int, int, int, int, int, hipStream_t);
int ca_conv_fwd_ex(const bf16_t*, const bf16_t*, bf16_t*, int, int, int, int, int, int, int, int, int, int, int,
                   const float*, int, hipStream_t);
int ca_conv_fwd(const bf16_t*, const bf16_t*, bf16_t*, int, int, int, int, int, int, int, int, int, int, int, float*,
                hipStream_t);
int ca_conv_dgrad(const bf16_t*, const bf16_t*, bf16_t*, int, int, int, int, int, int, int, int, int, int, int, float,
                  hipStream_t, int);
int ca_conv_wgrad(const bf16_t*, const bf16_t*, void*, int, float, int, int, int, int, int, int, int, int, int, int,
                  int, int, float*, hipStream_t);
int ca_splitk_reduce(const float*, int, long, void*, int, float, hipStream_t);
int ca_grad_finalize_multi(const uint64_t*, const float*, int, hipStream_t);
int ca_cls_head_max_labels();
int ca_cls_head_fwd(const bf16_t*, long, const float*, const float*, float*, int, int, int, float, uint64_t,
                    hipStream_t);
int ca_cls_head_bwd(const float*, const bf16_t*, long, const float*, bf16_t*, float*, float*, int, int, int, float,
                    uint64_t, hipStream_t);
int ca_gemm_splitk(int, const bf16_t*, long, const bf16_t*, long, void*, int, float, int, int, int, int, float*,
                   hipStream_t);
int ca_gemm_splitk_effective(int, int);
int ca_gemm_ex(int, const bf16_t*, long, const bf16_t*, long, bf16_t*, long, int, int, int, float*, float, const float*,
               int, bf16_t*, const bf16_t*, long, hipStream_t);
long ca_ln_workspace_floats(long, int);
int ca_ln_fwd(const bf16_t*, const bf16_t*, const float*, const float*, bf16_t*, bf16_t*, float*, float*, long, int,
              float, float, uint64_t, float, uint64_t, const float*, hipStream_t);
int ca_ln_bwd(const bf16_t*, const bf16_t*, const float*, const float*, const float*, bf16_t*, bf16_t*, float*, float*,
              int, float*, long, int, float, uint64_t, float, uint64_t, hipStream_t, float*);
long ca_colsum_workspace_floats(long, int);
int ca_colsum(const bf16_t*, long, int, long, float*, int, float*, hipStream_t);
int ca_act_grad(const bf16_t*, long, int, const bf16_t*, bf16_t*, long, int, int, hipStream_t);
int ca_pad_cols(const void*, long, int, void*, int, long, long, int, hipStream_t);
int ca_slice_acc(const float*, long, void*, int, long, int, hipStream_t);
int ca_pad_cols_multi(const long*, int, hipStream_t);
int ca_splitk_bias_act(const float*, int, long, int, const float*, int, bf16_t*, hipStream_t);
int ca_embed_sum(const int32_t*, const int32_t*, const float*, const float*, const float*, bf16_t*, long, int, int, int,
                 hipStream_t);
int ca_embed_bwd(const bf16_t*, const int32_t*, const int32_t*, float*, float*, float*, long, int, int, int, int, int,
                 int, float*, unsigned*, hipStream_t);
int ca_dropout(const bf16_t*, bf16_t*, long, float, uint64_t, hipStream_t);
int ca_dropout_mask(uint8_t*, long, long, float, uint64_t, hipStream_t);
int ca_attn_fwd(const bf16_t*, bf16_t*, float*, const int*, int, int, int, float, float, uint64_t, hipStream_t);
int ca_attn_bwd(const bf16_t*, const bf16_t*, const bf16_t*, const float*, float*, bf16_t*, const int*, int, int, int,
                float, float, uint64_t, hipStream_t);
}

#define P(T, x) reinterpret_cast<T>(static_cast<uintptr_t>(x))
#define S(x) reinterpret_cast<hipStream_t>(static_cast<uintptr_t>(x))

static void check(int rc, const char* what) {
  if (rc != 0) {
    std::string msg = std::string(what) + " failed: ";
    if (rc > 0) msg += hipGetErrorString(static_cast<hipError_t>(rc));
    else if (rc == -3)
      msg += "an operand window of one GEMM block exceeds the 2 GiB reach of the buffer loads (split the batch or K)";
    else msg += "invalid arguments (code " + std::to_string(rc) + ")";
    throw std::runtime_error(msg);
  }
}

typedef unsigned long long u64;

// dst waits for everything queued on src so far: a record / wait pair on a pooled event (no
// Python Event object per fork -- runtime/side_stream.py SideWork).  A wait binds to the
// record that precedes it, so an event is reusable as soon as its wait is enqueued; the ring
// only keeps concurrent callers (autograd threads) off each other's event.
static int stream_wait(u64 dst, u64 src) {
  static hipEvent_t ring[16];
  static std::atomic<int> next{0};
  static std::once_flag once;
  static hipError_t init_err = hipSuccess;
  std::call_once(once, [] {
    for (auto& e : ring) {
      const hipError_t rc = hipEventCreateWithFlags(&e, hipEventDisableTiming);
      if (rc != hipSuccess) init_err = rc;
    }
  });
  if (init_err != hipSuccess) return (int)init_err;
  hipEvent_t e = ring[next.fetch_add(1) & 15];
  hipError_t rc = hipEventRecord(e, S(src));
  if (rc == hipSuccess) rc = hipStreamWaitEvent(S(dst), e, 0);
  return (int)rc;
}

PYBIND11_MODULE(_C, m) {
  m.doc() = "cloud_amd gfx950 HIP kernels";
  m.attr("ARCH") = "gfx950";

  m.def("stream_wait", [](u64 dst, u64 src) { check(stream_wait(dst, src), "stream_wait"); },
        "dst waits for the work queued on src so far (pooled event)");

  // hp: device hyper-parameter array (0 = use hv, passed by value); zero_g: fused zero_grad
  m.def("sgd_step", [](u64 p, u64 g, int gbf, u64 mom, u64 p16, u64 hp, const std::vector<float>& hv, long n,
                       int nesterov, int zero_g, u64 s) {
    check(ca_sgd_step(P(float*, p), P(void*, g), gbf, P(float*, mom), P(bf16_t*, p16), P(const float*, hp),
                      hv.empty() ? nullptr : hv.data(), n, nesterov, zero_g, S(s)), "sgd_step");
  });
  m.def("adam_step", [](u64 p, u64 g, int gbf, u64 mm, u64 vv, u64 p16, u64 hp, const std::vector<float>& hv, long n,
                        int decoupled, int zero_g, u64 s) {
    check(ca_adam_step(P(float*, p), P(void*, g), gbf, P(float*, mm), P(float*, vv), P(bf16_t*, p16),
                       P(const float*, hp), hv.empty() ? nullptr : hv.data(), n, decoupled, zero_g, S(s)), "adam_step");
  });
  m.def("rmsprop_step", [](u64 p, u64 g, int gbf, u64 ms, u64 buf, u64 p16, u64 hp, const std::vector<float>& hv,
                           long n, int zero_g, u64 s) {
    check(ca_rmsprop_step(P(float*, p), P(void*, g), gbf, P(float*, ms), P(float*, buf), P(bf16_t*, p16),
                          P(const float*, hp), hv.empty() ? nullptr : hv.data(), n, zero_g, S(s)), "rmsprop_step");
  });
  m.def("sumsq", [](u64 g, int gbf, long n, u64 out, u64 s) {
    check(ca_sumsq(P(const void*, g), gbf, n, P(float*, out), S(s)), "sumsq");
  });
  m.def("scale", [](u64 g, int gbf, long n, u64 sc, u64 s) {
    check(ca_scale(P(void*, g), gbf, n, P(const float*, sc), S(s)), "scale");
  });
  m.def("bn_workspace_floats", [](long M, int C) { return ca_bn_workspace_floats(M, C); });
  m.def("bn_fwd", [](u64 x, u64 res, u64 y, long M, int C, u64 gamma, u64 beta, float eps, float momentum,
                     u64 rm, u64 rv, u64 sm, u64 sr, u64 ss, u64 ws, int relu, u64 mask, u64 s) {
    check(ca_bn_fwd(P(const bf16_t*, x), P(const bf16_t*, res), P(bf16_t*, y), M, C, P(const float*, gamma),
                    P(const float*, beta), eps, momentum, P(float*, rm), P(float*, rv), P(float*, sm), P(float*, sr),
                    P(float*, ss), P(float*, ws), relu, P(uint8_t*, mask), S(s)), "bn_fwd");
  });
  m.def("bn_fwd_partials", [](u64 x, u64 res, u64 y, long M, int C, u64 parts, int nparts, u64 gamma, u64 beta,
                              float eps, float momentum, u64 rm, u64 rv, u64 sm, u64 sr, u64 ss, int relu, u64 mask,
                              u64 gws, u64 s) {
    check(ca_bn_fwd_partials(P(const bf16_t*, x), P(const bf16_t*, res), P(bf16_t*, y), M, C, P(const float*, parts),
                             nparts, P(const float*, gamma), P(const float*, beta), eps, momentum, P(float*, rm),
                             P(float*, rv), P(float*, sm), P(float*, sr), P(float*, ss), relu, P(uint8_t*, mask),
                             P(float*, gws), S(s)),
          "bn_fwd_partials");
  });
  m.def("bn_apply", [](u64 x, u64 res, u64 y, long M, int C, u64 ss, int relu, u64 s) {
    check(ca_bn_apply(P(const bf16_t*, x), P(const bf16_t*, res), P(bf16_t*, y), M, C, P(const float*, ss), relu,
                      S(s)), "bn_apply");
  });
  m.def("bn_bwd", [](u64 dy, u64 y, u64 mask, u64 x, long M, int C, u64 gamma, u64 sm, u64 sr, u64 dx, u64 dres,
                     u64 dg, u64 db, u64 coef, u64 ws, int relu, u64 s) {
    check(ca_bn_bwd(P(const bf16_t*, dy), P(const bf16_t*, y), P(const uint8_t*, mask), P(const bf16_t*, x), M, C,
                    P(const float*, gamma),
                    P(const float*, sm), P(const float*, sr), P(bf16_t*, dx), P(bf16_t*, dres), P(float*, dg),
                    P(float*, db), P(float*, coef), P(float*, ws), relu, S(s)), "bn_bwd");
  });
  m.def("bn_bwd_partials", [](u64 dy, u64 y, u64 mask, u64 x, long M, int C, u64 parts, int nparts, u64 gamma,
                              u64 sm, u64 sr, u64 dx, u64 dres, u64 dg, u64 db, u64 coef, u64 gws, int relu, u64 s) {
    check(ca_bn_bwd_partials(P(const bf16_t*, dy), P(const bf16_t*, y), P(const uint8_t*, mask), P(const bf16_t*, x), M,
                             C, P(const float*, parts), nparts, P(const float*, gamma), P(const float*, sm),
                             P(const float*, sr), P(bf16_t*, dx), P(bf16_t*, dres), P(float*, dg), P(float*, db),
                             P(float*, coef), P(float*, gws), relu, S(s)),
          "bn_bwd_partials");
  });
  m.def("gemm_bf16_bnstats", [](int layout, u64 A, long lda, u64 B, long ldb, u64 C, long ldc, int M, int N, int K,
                                float beta, u64 z, u64 mask, u64 stats, u64 s) {
    check(ca_gemm_bf16_bnstats(layout, P(const bf16_t*, A), lda, P(const bf16_t*, B), ldb, P(bf16_t*, C), ldc, M, N, K,
                               beta, P(const bf16_t*, z), P(const uint8_t*, mask), P(float*, stats), S(s)),
          "gemm_bf16_bnstats");
  });
  m.def("dgrad_gemm", [](int layout, u64 A, long lda, u64 B, long ldb, u64 C, long ldc, int M, int N, int K,
                         float beta, u64 res, u64 res_mask, u64 z, u64 mask, u64 stats, u64 s, u64 z2, u64 stats2,
                         int par_s, int par_h, int par_w) {
    check(ca_dgrad_gemm(layout, P(const bf16_t*, A), lda, P(const bf16_t*, B), ldb, P(bf16_t*, C), ldc, M, N, K, beta,
                        P(const bf16_t*, res), P(const uint8_t*, res_mask), P(const bf16_t*, z),
                        P(const uint8_t*, mask), P(float*, stats), S(s), P(const bf16_t*, z2), P(float*, stats2), par_s,
                        par_h, par_w),
          "dgrad_gemm");
  }, py::arg("layout"), py::arg("A"), py::arg("lda"), py::arg("B"), py::arg("ldb"), py::arg("C"), py::arg("ldc"),
        py::arg("M"), py::arg("N"), py::arg("K"), py::arg("beta"), py::arg("res"), py::arg("res_mask"), py::arg("z"),
        py::arg("mask"), py::arg("stats"), py::arg("s"), py::arg("z2") = 0, py::arg("stats2") = 0,
        py::arg("par_s") = 0, py::arg("par_h") = 0, py::arg("par_w") = 0);
  m.def("gemm_xa", [](int layout, int mode, u64 src0, u64 src1, u64 mask_in, u64 c0, u64 c1, u64 c2, u64 c3, u64 side,
                      u64 mask_out, long lda, u64 B, long ldb, u64 C, long ldc, int M, int N, int K, float beta,
                      u64 res, u64 res_mask, u64 z, u64 mask, u64 stats, u64 z2, u64 stats2, u64 s) {
    check(ca_gemm_xa(layout, mode, P(const bf16_t*, src0), P(const bf16_t*, src1), P(const uint8_t*, mask_in),
                     P(const float*, c0), P(const float*, c1), P(const float*, c2), P(const float*, c3),
                     P(bf16_t*, side),
                     P(uint8_t*, mask_out), lda, P(const bf16_t*, B), ldb, P(bf16_t*, C), ldc, M, N, K, beta,
                     P(const bf16_t*, res), P(const uint8_t*, res_mask), P(const bf16_t*, z), P(const uint8_t*, mask),
                     P(float*, stats), P(const bf16_t*, z2), P(float*, stats2), S(s)),
          "gemm_xa");
  });
  m.def("gemm_xa_bwd_strided", [](u64 src0, u64 src1, u64 mask_in, u64 c0, u64 c1, u64 c2, u64 side, long lda, u64 B,
                                  long ldb, u64 C, long ldc, int M, int N, int K, int Nb, int H, int W, int stride,
                                  u64 s) {
    check(ca_gemm_xa_bwd_strided(P(const bf16_t*, src0), P(const bf16_t*, src1), P(const uint8_t*, mask_in),
                                 P(const float*, c0), P(const float*, c1), P(const float*, c2), P(bf16_t*, side), lda,
                                 P(const bf16_t*, B), ldb, P(bf16_t*, C), ldc, M, N, K, Nb, H, W, stride, S(s)),
          "gemm_xa_bwd_strided");
  });
  m.def("gemm_xa_dw", [](u64 src0, u64 src1, u64 mask_in, u64 c0, u64 c1, u64 c2, long lda, u64 B, long ldb, u64 C,
                         long ldc, int M, int N, int K, float beta, u64 res, u64 res_mask, u64 z, u64 mask, u64 stats,
                         u64 z2, u64 stats2, u64 y, long ldy, u64 dw, int dw_bf16, float dw_beta, u64 ws, int blocks,
                         u64 s) {
    const int g = ca_gemm_xa_dw(P(const bf16_t*, src0), P(const bf16_t*, src1), P(const uint8_t*, mask_in),
                                P(const float*, c0), P(const float*, c1), P(const float*, c2), lda,
                                P(const bf16_t*, B), ldb, P(bf16_t*, C), ldc, M, N, K, beta, P(const bf16_t*, res),
                                P(const uint8_t*, res_mask), P(const bf16_t*, z), P(const uint8_t*, mask),
                                P(float*, stats), P(const bf16_t*, z2), P(float*, stats2), P(const bf16_t*, y), ldy,
                                P(void*, dw), dw_bf16, dw_beta, P(float*, ws), blocks, S(s));
    check(g < 0 ? g : 0, "gemm_xa_dw");
    return g;
  });
  m.def("bn_fwd_partials_ex", [](u64 x, u64 res, u64 res_ss, u64 y, long M, int C, u64 parts, int nparts, u64 gamma,
                                 u64 beta, float eps, float momentum, u64 rm, u64 rv, u64 sm, u64 sr, u64 ss, int relu,
                                 u64 mask, u64 gws, u64 s) {
    check(ca_bn_fwd_partials_ex(P(const bf16_t*, x), P(const bf16_t*, res), P(const float*, res_ss), P(bf16_t*, y), M,
                                C, P(const float*, parts), nparts, P(const float*, gamma), P(const float*, beta), eps,
                                momentum, P(float*, rm), P(float*, rv), P(float*, sm), P(float*, sr), P(float*, ss),
                                relu, P(uint8_t*, mask), P(float*, gws), S(s)),
          "bn_fwd_partials_ex");
  });
  m.def("conv_dgrad_stat_tiles", [](int Nb, int H, int W, int sh, int sw) {
    return ca_conv_dgrad_stat_tiles(Nb, H, W, sh, sw);
  });
  m.def("conv_dgrad_stat_rows", [](int Nb, int H, int W, int Cin, int Cout, int KH, int KW, int sh, int sw, int ph,
                                   int pw, float beta) {
    return ca_conv_dgrad_stat_rows(Nb, H, W, Cin, Cout, KH, KW, sh, sw, ph, pw, beta);
  });
  m.def("conv_stat_rows", [](int Nb, int H, int W, int Cin, int Cout, int KH, int KW, int sh, int sw, int ph,
                             int pw) { return ca_conv_stat_rows(Nb, H, W, Cin, Cout, KH, KW, sh, sw, ph, pw); });
  m.def("conv_wgrad_splits", [](int Nb, int H, int W, int Cin, int Cout, int KH, int KW, int sh, int sw, int ph,
                                int pw, int fallback) {
    return ca_conv_wgrad_splits(Nb, H, W, Cin, Cout, KH, KW, sh, sw, ph, pw, fallback);
  });
  m.def("conv_dgrad_bnstats", [](u64 dy, u64 w, u64 dx, int Nb, int H, int W, int Cin, int Cout, int KH, int KW,
                                 int sh, int sw, int ph, int pw, float beta, u64 z, u64 mask, u64 stats, u64 s) {
    check(ca_conv_dgrad_bnstats(P(const bf16_t*, dy), P(const bf16_t*, w), P(bf16_t*, dx), Nb, H, W, Cin, Cout, KH, KW,
                                sh, sw, ph, pw, beta, P(const bf16_t*, z), P(const uint8_t*, mask), P(float*, stats),
                                S(s)),
          "conv_dgrad_bnstats");
  });
  m.def("u8_normalize", [](u64 x, u64 y, long n, std::vector<float> mean, std::vector<float> std_, u64 s) {
    if (mean.size() != std_.size() || mean.empty()) throw std::invalid_argument("u8_normalize: mean/std size");
    check(ca_u8_normalize(P(const uint8_t*, x), P(bf16_t*, y), n, (int)mean.size(), mean.data(), std_.data(), S(s)),
          "u8_normalize");
  });
  m.def("stem_s2d", [](u64 x, u64 y, int N, int H, int W, int C, int Hs, int Ws, int pad, u64 s) {
    check(ca_stem_s2d(P(const bf16_t*, x), P(bf16_t*, y), N, H, W, C, Hs, Ws, pad, S(s)), "stem_s2d");
  });
  m.def("softmax_xent", [](u64 z, int zbf, u64 labels, int B, int C, float gscale, float ls, u64 loss, u64 correct,
                           u64 dz, u64 s) {
    check(ca_softmax_xent(P(const void*, z), zbf, P(const int64_t*, labels), B, C, gscale, ls, P(float*, loss),
                          P(float*, correct), P(void*, dz), S(s)), "softmax_xent");
  });
  m.def("softmax_xent_batch", [](u64 z, long ldz, int bf, u64 labels, int B, int C, float gs, float ls, u64 mean, u64 correct,
                                 u64 dz, u64 acc, float acc_w, u64 s) {
    check(ca_softmax_xent_batch(P(const void*, z), ldz, bf, P(const int64_t*, labels), B, C, gs, ls, P(float*, mean),
                                P(float*, correct), P(void*, dz), P(float*, acc), acc_w, S(s)), "softmax_xent_batch");
  });
  m.def("maxpool_fwd", [](u64 x, u64 y, u64 idx, int N, int H, int W, int C, int OH, int OW, int k, int st, int p,
                          u64 s) {
    check(ca_maxpool_fwd(P(const bf16_t*, x), P(bf16_t*, y), P(uint8_t*, idx), N, H, W, C, OH, OW, k, st, p, S(s)),
          "maxpool_fwd");
  });
  m.def("maxpool_bwd", [](u64 dy, u64 idx, u64 dx, int N, int H, int W, int C, int OH, int OW, int k, int st, int p,
                          u64 s) {
    check(ca_maxpool_bwd(P(const bf16_t*, dy), P(const uint8_t*, idx), P(bf16_t*, dx), N, H, W, C, OH, OW, k, st, p,
                         S(s)), "maxpool_bwd");
  });
  m.def("gap_fwd", [](u64 x, u64 y, int ybf, int N, int HW, int C, u64 s) {
    check(ca_gap_fwd(P(const bf16_t*, x), P(void*, y), ybf, N, HW, C, S(s)), "gap_fwd");
  });
  m.def("gemm_bf16", [](int layout, u64 A, long lda, u64 B, long ldb, u64 C, long ldc, int M, int N, int K,
                        u64 stats, float beta, u64 s) {
    check(ca_gemm_bf16(layout, P(const bf16_t*, A), lda, P(const bf16_t*, B), ldb, P(bf16_t*, C), ldc, M, N, K,
                       P(float*, stats), beta, S(s)), "gemm_bf16");
  });
  m.def("conv_fwd", [](u64 x, u64 w, u64 y, int Nb, int H, int W, int Cin, int Cout, int KH, int KW, int sh, int sw,
                       int ph, int pw, u64 stats, u64 s) {
    check(ca_conv_fwd(P(const bf16_t*, x), P(const bf16_t*, w), P(bf16_t*, y), Nb, H, W, Cin, Cout, KH, KW, sh, sw, ph,
                      pw, P(float*, stats), S(s)), "conv_fwd");
  });
  m.def("bn_relu_maxpool_s2k3", [](u64 z, u64 ss, u64 y, u64 idx, int N, int H, int W, int C, int OH, int OW,
                                   u64 s) {
    check(ca_bn_relu_maxpool_s2k3(P(const bf16_t*, z), P(const float*, ss), P(bf16_t*, y), P(uint8_t*, idx), N, H, W,
                                  C, OH, OW, S(s)), "bn_relu_maxpool_s2k3");
  });
  m.def("gemm_set_core", [](int kind) { return ca_gemm_set_core(kind); });
  m.def("gemm_set_xa_n256", [](int mode) { return ca_gemm_set_xa_n256(mode); });
  m.def("gemm_set_streamk", [](int mode) { return ca_gemm_set_streamk(mode); });
  m.def("experimental_built", []() { return ca_gemm_experimental_built() != 0; });
  m.def("maxpool_bnstats_parts", [](int N, int H, int W, int C) { return ca_maxpool_bnstats_parts(N, H, W, C); });
  m.def("maxpool_bwd_s2k3_bnstats", [](u64 dy, u64 yp, u64 idx, u64 z, u64 g, u64 part, int N, int H, int W, int C,
                                       int OH, int OW, u64 s) {
    check(ca_maxpool_bwd_s2k3_bnstats(P(const bf16_t*, dy), P(const bf16_t*, yp), P(const uint8_t*, idx),
                                      P(const bf16_t*, z), P(bf16_t*, g), P(float*, part), N, H, W, C, OH, OW, S(s)),
          "maxpool_bwd_s2k3_bnstats");
  });
  m.def("maxpool_bwd_s2k3_bnapply", [](u64 dy, u64 yp, u64 idx, u64 z, u64 coef, u64 dz, int N, int H, int W, int C,
                                       int OH, int OW, u64 s) {
    check(ca_maxpool_bwd_s2k3_bnapply(P(const bf16_t*, dy), P(const bf16_t*, yp), P(const uint8_t*, idx),
                                      P(const bf16_t*, z), P(const float*, coef), P(bf16_t*, dz), N, H, W, C, OH, OW,
                                      S(s)),
          "maxpool_bwd_s2k3_bnapply");
  });
  m.def("conv_fwd_ex", [](u64 x, u64 w, u64 y, int Nb, int H, int W, int Cin, int Cout, int KH, int KW, int sh,
                          int sw, int ph, int pw, u64 bias, int act, u64 s) {
    check(ca_conv_fwd_ex(P(const bf16_t*, x), P(const bf16_t*, w), P(bf16_t*, y), Nb, H, W, Cin, Cout, KH, KW, sh, sw,
                         ph, pw, P(const float*, bias), act, S(s)), "conv_fwd_ex");
  });
  m.def("conv_dgrad", [](u64 dy, u64 w, u64 dx, int Nb, int H, int W, int Cin, int Cout, int KH, int KW, int sh,
                         int sw, int ph, int pw, float beta, u64 s, int skip_empty) {
    check(ca_conv_dgrad(P(const bf16_t*, dy), P(const bf16_t*, w), P(bf16_t*, dx), Nb, H, W, Cin, Cout, KH, KW, sh, sw,
                        ph, pw, beta, S(s), skip_empty), "conv_dgrad");
  }, py::arg("dy"), py::arg("w"), py::arg("dx"), py::arg("Nb"), py::arg("H"), py::arg("W"), py::arg("Cin"),
        py::arg("Cout"), py::arg("KH"), py::arg("KW"), py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"),
        py::arg("beta"), py::arg("s"), py::arg("skip_empty") = 0);
  m.def("conv_wgrad", [](u64 dy, u64 x, u64 dw, int dw_bf16, float beta, int Nb, int H, int W, int Cin, int Cout,
                         int KH, int KW, int sh, int sw, int ph, int pw, int splits, u64 ws, u64 s) {
    check(ca_conv_wgrad(P(const bf16_t*, dy), P(const bf16_t*, x), P(void*, dw), dw_bf16, beta, Nb, H, W, Cin, Cout,
                        KH, KW, sh, sw, ph, pw, splits, P(float*, ws), S(s)), "conv_wgrad");
  });
  // jobs: rows of 12 u64 {kind, src, nparts, stride, n, out0, out1, out2, out_bf16, accumulate, 0, 0}
  m.def("grad_finalize_multi", [](const std::vector<uint64_t>& jobs, const std::vector<float>& betas, u64 s) {
    const int n = (int)betas.size();
    if ((long)jobs.size() != 12L * n) throw std::runtime_error("grad_finalize_multi: 12 fields per job");
    check(ca_grad_finalize_multi(jobs.data(), betas.data(), n, S(s)), "grad_finalize_multi");
  });
  m.def("cls_head_max_labels", []() { return ca_cls_head_max_labels(); });
  m.def("cls_head_fwd", [](u64 pooled, long ldp, u64 wc, u64 bc, u64 logits, int B, int C, int L, float p, u64 seed,
                           u64 s) {
    check(ca_cls_head_fwd(P(const bf16_t*, pooled), ldp, P(const float*, wc), P(const float*, bc), P(float*, logits),
                          B, C, L, p, seed, S(s)), "cls_head_fwd");
  });
  m.def("cls_head_bwd", [](u64 dl, u64 pooled, long ldp, u64 wc, u64 dpre, u64 gwc, u64 gbc, int B, int C, int L,
                           float p, u64 seed, u64 s) {
    check(ca_cls_head_bwd(P(const float*, dl), P(const bf16_t*, pooled), ldp, P(const float*, wc), P(bf16_t*, dpre),
                          P(float*, gwc), P(float*, gbc), B, C, L, p, seed, S(s)), "cls_head_bwd");
  });
  m.def("splitk_reduce", [](u64 ws, int splits, long MN, u64 out, int out_bf16, float beta, u64 s) {
    check(ca_splitk_reduce(P(const float*, ws), splits, MN, P(void*, out), out_bf16, beta, S(s)), "splitk_reduce");
  });
  m.def("gemm_splitk", [](int layout, u64 A, long lda, u64 B, long ldb, u64 out, int out_bf16, float beta, int M,
                          int N, int K, int splits, u64 ws, u64 s) {
    check(ca_gemm_splitk(layout, P(const bf16_t*, A), lda, P(const bf16_t*, B), ldb, P(void*, out), out_bf16, beta,
                         M, N, K, splits, P(float*, ws), S(s)), "gemm_splitk");
  });
  m.def("gemm_stat_rows", [](int M, int N, int K, long lda, long ldb, long ldc) {
    return ca_gemm_stat_rows(M, N, K, lda, ldb, ldc);
  });
  m.def("gemm_splitk_effective", [](int K, int splits) { return ca_gemm_splitk_effective(K, splits); });
  m.def("gap_bwd", [](u64 dy, int dybf, u64 dx, int N, int HW, int C, u64 s) {
    check(ca_gap_bwd(P(const void*, dy), dybf, P(bf16_t*, dx), N, HW, C, S(s)), "gap_bwd");
  });
  m.def("gmp_fwd", [](u64 x, u64 y, u64 cnt, int N, int HW, int C, u64 s) {
    check(ca_gmp_fwd(P(const bf16_t*, x), P(bf16_t*, y), P(float*, cnt), N, HW, C, S(s)), "gmp_fwd");
  });
  m.def("gmp_bwd", [](u64 dy, int dy_bf16, u64 x, u64 y, u64 cnt, u64 dx, int N, int HW, int C, u64 s) {
    check(ca_gmp_bwd(P(const void*, dy), dy_bf16, P(const bf16_t*, x), P(const bf16_t*, y), P(const float*, cnt),
                     P(bf16_t*, dx), N, HW, C, S(s)), "gmp_bwd");
  });
  m.def("gemm_ex", [](int layout, u64 A, long lda, u64 B, long ldb, u64 C, long ldc, int M, int N, int K, u64 stats,
                      float beta, u64 bias, int act, u64 preact, u64 dact_src, long ld_aux, u64 s) {
    check(ca_gemm_ex(layout, P(const bf16_t*, A), lda, P(const bf16_t*, B), ldb, P(bf16_t*, C), ldc, M, N, K,
                     P(float*, stats), beta, P(const float*, bias), act, P(bf16_t*, preact), P(const bf16_t*, dact_src),
                     ld_aux, S(s)), "gemm_ex");
  });
  m.def("ln_workspace_floats", [](long M, int C) { return ca_ln_workspace_floats(M, C); });
  m.def("ln_fwd", [](u64 x, u64 res, u64 g, u64 b, u64 y, u64 h, u64 mu, u64 rs, long M, int C, float eps, float p_in,
                     u64 seed_in, float p_out, u64 seed_out, u64 s, u64 xb) {
    check(ca_ln_fwd(P(const bf16_t*, x), P(const bf16_t*, res), P(const float*, g), P(const float*, b), P(bf16_t*, y),
                    P(bf16_t*, h), P(float*, mu), P(float*, rs), M, C, eps, p_in, seed_in, p_out, seed_out,
                    P(const float*, xb), S(s)),
          "ln_fwd");
  });
  m.def("ln_bwd", [](u64 dy, u64 h, u64 mu, u64 rs, u64 g, u64 dh, u64 dx, u64 dg, u64 db, int acc, u64 ws, long M,
                     int C, float p_in, u64 seed_in, float p_out, u64 seed_out, u64 s, u64 dsum) {
    check(ca_ln_bwd(P(const bf16_t*, dy), P(const bf16_t*, h), P(const float*, mu), P(const float*, rs),
                    P(const float*, g), P(bf16_t*, dh), P(bf16_t*, dx), P(float*, dg), P(float*, db), acc,
                    P(float*, ws), M, C, p_in, seed_in, p_out, seed_out, S(s), P(float*, dsum)), "ln_bwd");
  }, py::arg("dy"), py::arg("h"), py::arg("mu"), py::arg("rs"), py::arg("g"), py::arg("dh"), py::arg("dx"),
        py::arg("dg"), py::arg("db"), py::arg("acc"), py::arg("ws"), py::arg("M"), py::arg("C"), py::arg("p_in"),
        py::arg("seed_in"), py::arg("p_out"), py::arg("seed_out"), py::arg("s"), py::arg("dsum") = 0);
  m.def("pad_cols", [](u64 in, long ld, int cols, u64 out, int cols_out, long rows, long rows_out, int eb, u64 s) {
    check(ca_pad_cols(P(const void*, in), ld, cols, P(void*, out), cols_out, rows, rows_out, eb, S(s)), "pad_cols");
  });
  m.def("splitk_bias_act", [](u64 ws, int splits, long M, int N, u64 bias, int act, u64 out, u64 s) {
    check(ca_splitk_bias_act(P(const float*, ws), splits, M, N, P(const float*, bias), act, P(bf16_t*, out), S(s)),
          "splitk_bias_act");
  });
  m.def("pad_cols_multi", [](std::vector<long> jobs, u64 s) {
    check(ca_pad_cols_multi(jobs.data(), (int)(jobs.size() / 8), S(s)), "pad_cols_multi");
  });
  m.def("slice_acc", [](u64 in, long ld_in, u64 out, int out_bf16, long rows, int cols, u64 s) {
    check(ca_slice_acc(P(const float*, in), ld_in, P(void*, out), out_bf16, rows, cols, S(s)), "slice_acc");
  });
  m.def("act_grad", [](u64 dy, long ld_dy, int N, u64 src, u64 out, long M, int Np, int act, u64 s) {
    check(ca_act_grad(P(const bf16_t*, dy), ld_dy, N, P(const bf16_t*, src), P(bf16_t*, out), M, Np, act, S(s)),
          "act_grad");
  });
  m.def("colsum_workspace_floats", [](long M, int N) { return ca_colsum_workspace_floats(M, N); });
  m.def("colsum", [](u64 x, long M, int N, long ld, u64 out, int acc, u64 ws, u64 s) {
    check(ca_colsum(P(const bf16_t*, x), M, N, ld, P(float*, out), acc, P(float*, ws), S(s)), "colsum");
  });
  m.def("embed_sum", [](u64 ids, u64 tts, u64 word, u64 pos, u64 type, u64 h, long M, int S_, int C, int po, u64 s) {
    check(ca_embed_sum(P(const int32_t*, ids), P(const int32_t*, tts), P(const float*, word), P(const float*, pos),
                       P(const float*, type), P(bf16_t*, h), M, S_, C, po, S(s)), "embed_sum");
  });
  // returns 1 when a gradient took the order-dependent float-atomic path
  m.def("embed_bwd", [](u64 dh, u64 ids, u64 tts, u64 dw, u64 dp, u64 dt, long M, int S_, int C, int T, int po,
                        int pad_id, int V, u64 tws, u64 tk, u64 s) {
    const int r = ca_embed_bwd(P(const bf16_t*, dh), P(const int32_t*, ids), P(const int32_t*, tts), P(float*, dw),
                               P(float*, dp), P(float*, dt), M, S_, C, T, po, pad_id, V, P(float*, tws),
                               P(unsigned*, tk), S(s));
    if (r < 0) check(r, "embed_bwd");
    return r;
  });
  m.def("dropout", [](u64 x, u64 y, long n, float p, u64 seed, u64 s) {
    check(ca_dropout(P(const bf16_t*, x), P(bf16_t*, y), n, p, seed, S(s)), "dropout");
  });
  m.def("dropout_mask", [](u64 m_, long n, long base, float p, u64 seed, u64 s) {
    check(ca_dropout_mask(P(uint8_t*, m_), n, base, p, seed, S(s)), "dropout_mask");
  });
  m.def("attn_fwd", [](u64 qkv, u64 ctx, u64 lse, u64 klen, int B, int S_, int H, float scale, float p, u64 seed,
                       u64 s) {
    check(ca_attn_fwd(P(const bf16_t*, qkv), P(bf16_t*, ctx), P(float*, lse), P(const int*, klen), B, S_, H, scale, p,
                      seed, S(s)), "attn_fwd");
  });
  m.def("attn_bwd", [](u64 qkv, u64 out, u64 dout, u64 lse, u64 dvec, u64 dqkv, u64 klen, int B, int S_, int H,
                       float scale, float p, u64 seed, u64 s) {
    check(ca_attn_bwd(P(const bf16_t*, qkv), P(const bf16_t*, out), P(const bf16_t*, dout), P(const float*, lse),
                      P(float*, dvec), P(bf16_t*, dqkv), P(const int*, klen), B, S_, H, scale, p, seed, S(s)),
          "attn_bwd");
  });
}
