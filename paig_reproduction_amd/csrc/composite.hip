// Composite entry points of SURVEY §8 B3 over the library's own kernels
// (host code): the localiser's dense layers and the velocity encoder +
// physics rollout, each as one call each way, for hosts that bind the C ABI
// without this package's Python engine (which calls the parts itself so its
// probes time each launch and its slab rows join the step's one batched
// reduction).  The same launches in the same order as the engine.
#include "common.h"

#define COMP_HIP(call)                                                  \
  do {                                                                  \
    const hipError_t _e = (call);                                       \
    if (_e != hipSuccess) {                                             \
      paig_set_error("%s: %s", __func__, hipGetErrorString(_e));        \
      return (int)_e;                                                   \
    }                                                                   \
  } while (0)
#define COMP_RC(call)          \
  do {                         \
    const int _rc = (call);    \
    if (_rc != 0) return _rc;  \
  } while (0)

namespace {
size_t c256(size_t b) { return (b + 255) & ~(size_t)255; }

// localiser workspace (bytes): [gemm slabs | W2^T] forward, [dh2 | dh1 |
// head slab | gemm workspace] backward (the two share the space)
size_t loc_fwd_bytes(int KF, int n1, int IN, int math) {
  return c256(paig_gemm_parts_size(KF, IN, n1, math) * 4) + c256((size_t)IN * IN * 4);
}
size_t loc_gemm_ws(int KF, int n1, int IN) {
  size_t w = paig_gemm_workspace(IN, IN, KF);
  w = w > paig_gemm_workspace(IN, n1, KF) ? w : paig_gemm_workspace(IN, n1, KF);
  w = w > paig_gemm_workspace(KF, n1, IN) ? w : paig_gemm_workspace(KF, n1, IN);
  return w;
}
size_t loc_bwd_bytes(int KF, int n1, int IN) {
  return 2 * c256((size_t)KF * IN * 4) + c256((size_t)paig_head_l2_bwd_blocks(KF) * (2 * IN + 2) * 4) +
         c256(loc_gemm_ws(KF, n1, IN) * 4);
}
}  // namespace

extern "C" {

size_t paig_localiser_workspace(int F, int K, int n1, int IN, int math) {
  const int KF = K * F;
  if (KF <= 0 || n1 <= 0 || IN <= 0) return 0;
  const size_t a = loc_fwd_bytes(KF, n1, IN, math), b = loc_bwd_bytes(KF, n1, IN);
  return a > b ? a : b;
}

int paig_localiser_fwd(const float* x1, const float* W1, const float* b1, const float* W2, const float* b2,
                       const float* W3, const float* b3, float* h1, float* h2, float* h3, float* pos, int F, int K,
                       int n1, int IN, float half, int math, void* ws, size_t ws_bytes, void* stream) {
  const int KF = K * F;
  PAIG_REQUIRE(KF > 0 && n1 > 0 && ws && ws_bytes >= paig_localiser_workspace(F, K, n1, IN, math),
               "paig_localiser_fwd: F=%d K=%d n1=%d, workspace %zu bytes", F, K, n1, ws_bytes);
  char* base = static_cast<char*>(ws);
  float* part = reinterpret_cast<float*>(base);
  float* w2t = reinterpret_cast<float*>(base + c256(paig_gemm_parts_size(KF, IN, n1, math) * 4));
  const int S = paig_gemm_parts(0, 1, KF, IN, n1, x1, n1, W1, n1, part, paig_gemm_parts_size(KF, IN, n1, math), math,
                                stream);
  if (S <= 0) return S < 0 ? S : PAIG_E_SHAPE;
  return paig_dense_tail_fwd(part, S, b1, h1, W2, w2t, b2, h2, W3, b3, h3, pos, F, K, IN, half, stream);
}

int paig_localiser_bwd(const float* dpos, const float* x1, const float* h1, const float* h2, const float* h3,
                       const float* W1, const float* W2, const float* W3, float* dl1, float* dl2, float* dl3,
                       float* dx1, int F, int K, int n1, int IN, float half, int math, void* ws, size_t ws_bytes,
                       void* stream) {
  const int KF = K * F;
  PAIG_REQUIRE(KF > 0 && n1 > 0 && ws && ws_bytes >= paig_localiser_workspace(F, K, n1, IN, math) && dl1 && dl2 &&
                   dl3,
               "paig_localiser_bwd: F=%d K=%d n1=%d, workspace %zu bytes, or a null gradient", F, K, n1, ws_bytes);
  char* base = static_cast<char*>(ws);
  float* dh2 = reinterpret_cast<float*>(base);
  float* dh1 = reinterpret_cast<float*>(base + c256((size_t)KF * IN * 4));
  float* hslab = reinterpret_cast<float*>(base + 2 * c256((size_t)KF * IN * 4));
  float* gws = reinterpret_cast<float*>(base + 2 * c256((size_t)KF * IN * 4) +
                                        c256((size_t)paig_head_l2_bwd_blocks(KF) * (2 * IN + 2) * 4));
  const size_t ngws = loc_gemm_ws(KF, n1, IN);
  // the position head + l2's data gradient (l1's ReLU' applied)
  COMP_RC(paig_head_l2_bwd(h2, h3, dpos, W3, dh2, hslab, F, K, IN, half, nullptr, nullptr, 0, 0, 0, 0, W2, h1, dh1, 0,
                           nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                           nullptr, stream));
  // l2 / l1 weight gradients (bias gradients = the row sums of dY^T), l1's data gradient
  COMP_RC(paig_gemm_ex(1, 0, IN, IN, KF, 1.f, dh2, IN, h1, IN, 0.f, dl2, IN, nullptr, 0, 0, nullptr, 0,
                       dl2 + (size_t)IN * IN, gws, ngws, math, stream));
  COMP_RC(paig_gemm_ex(1, 0, IN, n1, KF, 1.f, dh1, IN, x1, n1, 0.f, dl1, n1, nullptr, 0, 0, nullptr, 0,
                       dl1 + (size_t)IN * n1, gws, ngws, math, stream));
  if (dx1)
    COMP_RC(paig_gemm_ex(0, 0, KF, n1, IN, 1.f, dh1, IN, W1, n1, 0.f, dx1, n1, nullptr, 0, 0, nullptr, 0, nullptr,
                         gws, ngws, math, stream));
  const float* src[1] = {hslab};
  const int nb[1] = {paig_head_l2_bwd_blocks(KF)}, len[1] = {2 * IN + 2};
  float* dst[1] = {dl3};
  return paig_slab_reduce_multi(1, src, nb, len, dst, 0, stream);
}

size_t paig_velmlp_rollout_bwd_workspace(int B, int K, int S) {
  if (B <= 0 || K <= 0 || S <= 0) return 0;
  const int D = 2 * K, rows = K * B;
  return c256((size_t)B * D * 4) * 2 + c256((size_t)paig_rollout_bwd_blocks(B) * 2 * 8) +
         c256((size_t)rows * 2 * S * 4) + c256((size_t)paig_velmlp_bwd_blocks(rows) * paig_velmlp_slab_len(S) * 4);
}

int paig_velmlp_rollout_fwd(int cell, const float* pos, int B, int Te, int K, int S, const float* W0, const float* b0,
                            const float* W2, const float* b2, const float* W4, const float* b4, float* X, float* h1,
                            float* h2, float* vel0, const float* dt, const double* p0, const double* p1, float* pvs,
                            int R, void* stream) {
  PAIG_REQUIRE(B > 0 && K > 0 && S >= 1 && S <= Te && R > 0, "velmlp_rollout_fwd: B=%d K=%d S=%d Te=%d R=%d", B, K,
               S, Te, R);
  const int D = 2 * K;
  COMP_RC(paig_velmlp_fwd(pos, B, Te, K, S, W0, b0, W2, b2, W4, b4, X, h1, h2, vel0, stream));
  return paig_rollout_fwd(cell, pos + (size_t)(S - 1) * D, (long long)Te * D, vel0, dt, p0, p1, pvs, B, D, R, stream);
}

int paig_velmlp_rollout_bwd(int cell, const float* pvs, const float* dpos_roll, const float* dpvs, const float* dt,
                            const double* p0, const double* p1, const float* X, const float* h1, const float* h2,
                            const float* W0, const float* W2, const float* W4, float* dpos, float* dmlp,
                            double* gparam0, double* gparam1, int B, int Te, int K, int S, int R, void* ws,
                            size_t ws_bytes, void* stream) {
  PAIG_REQUIRE(B > 0 && K > 0 && S >= 1 && S <= Te && R > 0 && ws &&
                   ws_bytes >= paig_velmlp_rollout_bwd_workspace(B, K, S) && dpos && dmlp,
               "velmlp_rollout_bwd: B=%d K=%d S=%d Te=%d R=%d, workspace %zu bytes", B, K, S, Te, R, ws_bytes);
  const int D = 2 * K, rows = K * B;
  char* base = static_cast<char*>(ws);
  float* dpos0 = reinterpret_cast<float*>(base);
  float* dvel0 = reinterpret_cast<float*>(base + c256((size_t)B * D * 4));
  double* part = reinterpret_cast<double*>(base + 2 * c256((size_t)B * D * 4));
  float* dX = reinterpret_cast<float*>(base + 2 * c256((size_t)B * D * 4) +
                                       c256((size_t)paig_rollout_bwd_blocks(B) * 2 * 8));
  float* slab = reinterpret_cast<float*>(reinterpret_cast<char*>(dX) + c256((size_t)rows * 2 * S * 4));
  // the rollout adjoint (all R steps), then the velocity MLP's backward
  COMP_RC(paig_rollout_bwd(cell, pvs, dpos_roll, dpvs, dt, p0, p1, dpos0, dvel0, part, gparam0, gparam1, 0, B, D, R,
                           stream));
  COMP_RC(paig_velmlp_bwd(dvel0, X, h1, h2, W0, W2, W4, dX, slab, rows, S, stream));
  // d pos += the packed input gradient and d pos0 (step S-1)
  COMP_RC(paig_vel_unpack_add(dX, dpos0, dpos, B, Te, K, S, 0, stream));
  const float* src[1] = {slab};
  const int nb[1] = {paig_velmlp_bwd_blocks(rows)}, len[1] = {paig_velmlp_slab_len(S)};
  float* dst[1] = {dmlp};
  return paig_slab_reduce_multi(1, src, nb, len, dst, 0, stream);
}

}  // extern "C"
