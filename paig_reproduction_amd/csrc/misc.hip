// Small kernels of the step:
//   * VariableFromNetwork forward/backward (nn/network/blocks.py:311-322): the
//     decoder's template/content/background MLPs on a constant ones[1,10] input,
//     computed ONCE per step (the reference recomputes them on every one of the
//     R+1 decoder calls -- quirk Q12; the gradient is identical);
//   * loss reduction from per-frame SSE (nn/network/physics_models.py:119-142)
//     and its backward (per-frame loss weights, no dense dL/dframe);
//   * optimizers on the flat parameter buffer (nn/network/base.py:12-17:
//     RMSprop default, Adam, SGD, SGD+momentum; torch default hyper-params).
#include <math.h>
#include <stdarg.h>
#include <stdio.h>

#include "common.h"
#include "vfn.h"

static thread_local char g_err[512];

void paig_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

namespace {

using namespace paig_vfn;

__global__ void __launch_bounds__(256) vfn_fwd_k(VfnFwdTasks T) { vfn_fwd_block(T, blockIdx.x); }

// dy = d (raw) or d * s (1 - s), s = sigmoid(y) ; dW2 = dy h^T ; db2 = dy ;
// part[blk][j] = sum_{p in blk} W2[p][j] dy[p]
__global__ void __launch_bounds__(256) vfn_bwd1_k(VfnBwdTasks T) {
  const int k = task_of(T.blk0, T.n, blockIdx.x);
  const int bid = blockIdx.x - T.blk0[k];
  const float* __restrict__ d = T.d[k];
  const float* __restrict__ W2 = T.W2[k];
  float* __restrict__ dW2 = T.dW2[k];
  const int P = T.P[k], sig = T.sig[k];
  const int j = threadIdx.x;
  const int p0 = bid * VROWS;
  int p1 = p0 + VROWS;
  if (p1 > P) p1 = P;
  const float hj = j < VH ? T.h[k][j] : 0.f;
  // every load of the block's rows is issued before the first store (the
  // stores through T's pointers could alias them: loads interleaved with
  // stores ran one memory latency per row)
  float gr[VROWS], yv[VROWS], w2[VROWS];
#pragma unroll
  for (int r = 0; r < VROWS; ++r) {
    const int p = p0 + r < p1 ? p0 + r : p0;
    gr[r] = d[p];
    yv[r] = sig ? T.y[k][p] : 0.f;
    w2[r] = j < VH ? W2[(long long)p * VH + j] : 0.f;
  }
  float acc = 0.f;
#pragma unroll
  for (int r = 0; r < VROWS; ++r) {
    const int p = p0 + r;
    if (p >= p1) break;
    float g = gr[r];
    if (sig) {
      const float s = 1.f / (1.f + expf(-yv[r]));
      g = g * (s * (1.f - s));
    }
    if (j < VH) {
      dW2[(long long)p * VH + j] = g * hj;
      acc = fmaf(w2[r], g, acc);
    }
    if (j == 0) T.db2[k][p] = g;
  }
  if (j < VH) T.part[k][bid * VH + j] = acc;
}

// one 64-lane block per (instance, hidden unit j): dh[j] = sum of the
// partials, then the tanh' and the first layer's grads (input = ones)
__global__ void vfn_bwd2_k(VfnBwdTasks T) { vfn_bwd2_item(T, blockIdx.x, threadIdx.x); }

// losses: pred, extrap, recons (means of per-frame SSE)
__global__ void loss_reduce_k(const float* __restrict__ sse_rec, const float* __restrict__ sse_roll, int B, int Te,
                              int R, int pred, float ae, float* __restrict__ o_pred, float* __restrict__ o_ext,
                              float* __restrict__ o_rec) {
  __shared__ float red[3][16];   // one block of up to 1024 threads (16 waves)
  float a = 0.f, b = 0.f, c = 0.f;
  for (int i = threadIdx.x; i < B * R; i += blockDim.x) {
    const int t = i % R;
    if (t < pred) a += sse_roll[i];
    else b += sse_roll[i];
  }
  for (int i = threadIdx.x; i < B * Te; i += blockDim.x) c += sse_rec[i];
  a = wave_sum(a);
  b = wave_sum(b);
  c = wave_sum(c);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wv] = a;
    red[1][wv] = b;
    red[2][wv] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float s[3];
    const int nw = blockDim.x >> 6;
    for (int k = 0; k < 3; ++k) {
      s[k] = 0.f;
      for (int w = 0; w < nw; ++w) s[k] += red[k][w];
    }
    const float pl = s[0] / (float)(B * pred), rl = s[2] / (float)(B * Te);
    // train = pred (+= ae * recons, physics_models.py:137-141: a separate fp32
    // multiply then add, never contracted into an FMA)
    *o_pred = ae > 0.f ? __fadd_rn(pl, __fmul_rn(ae, rl)) : pl;
    *o_ext = (R - pred) > 0 ? s[1] / (float)(B * (R - pred)) : nanf("");
    *o_rec = rl;
  }
}

// per-frame loss weights from the loss adjoints (any may be null = 0);
// dpred is the adjoint of train = pred + ae * recons
__global__ void loss_bwd_k(const float* __restrict__ dpred, const float* __restrict__ dext,
                           const float* __restrict__ drec, float ae, float* __restrict__ wrec,
                           float* __restrict__ wroll, int B, int Te, int R, int pred) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < B * R; i += gridDim.x * blockDim.x)
    if (wroll) wroll[i] = loss_weight(2, i, dpred, dext, drec, ae, B, Te, R, pred);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < B * Te; i += gridDim.x * blockDim.x)
    if (wrec) wrec[i] = loss_weight(1, i, dpred, dext, drec, ae, B, Te, R, pred);
}

// per-frame SSE of dense frames vs targets (the unfused path, used when the
// loss is taken on frames that did not come from the current forward)
__global__ void __launch_bounds__(256) frame_sse_k(FView a, FView b, float* __restrict__ sse, int F, int n) {
  __shared__ float red[4];
  for (int f = blockIdx.x; f < F; f += gridDim.x) {
    const float* pa = a.frame(f);
    const float* pb = b.frame(f);
    float s = 0.f;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const float d = pb[i] - pa[i];
      s = fmaf(d, d, s);
    }
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) sse[f] = (red[0] + red[1]) + (red[2] + red[3]);
    __syncthreads();
  }
}

// dframe[f][i] = 2 * w[f] * (a - b)
__global__ void frame_sse_bwd_k(FView a, FView b, const float* __restrict__ w, float* __restrict__ da, int F, int n) {
  const long long tot = (long long)F * n;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < tot; i += (long long)gridDim.x * blockDim.x) {
    const int f = (int)(i / n), e = (int)(i % n);
    da[i] = 2.f * w[f] * (a.frame(f)[e] - b.frame(f)[e]);
  }
}

// ------------------------------------------------------------- optimizers ---
template <typename T>
__global__ void rmsprop_k(T* __restrict__ p, const T* __restrict__ g, T* __restrict__ sa, long long n, T lr, T alpha,
                          T eps) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const T gi = g[i];
    T s = sa[i] * alpha;
    s = s + (T(1) - alpha) * gi * gi;
    sa[i] = s;
    p[i] = p[i] - lr * gi / (sqrt(s) + eps);
  }
}

// RMSprop over both flat buffers in one launch: the fp32 parameters
// grid-stride, and block 0 also updates the few fp64 ones (the physics
// parameters) -- rmsprop_k's arithmetic in each precision
__global__ void rmsprop_mixed_k(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ sa, long long n,
                                float lr, float alpha, float eps, double* __restrict__ pd, const double* __restrict__ gd,
                                double* __restrict__ sd, long long nd, double lrd, double alphad, double epsd,
                                int vec) {
  if (blockIdx.x == 0)
    for (long long i = threadIdx.x; i < nd; i += blockDim.x) {
      const double gi = gd[i];
      double s = sd[i] * alphad;
      s = s + (1.0 - alphad) * gi * gi;
      sd[i] = s;
      pd[i] = pd[i] - lrd * gi / (sqrt(s) + epsd);
    }
  auto upd = [&](float pi, float gi, float si, float& po, float& so) __attribute__((always_inline)) {
    float s = si * alpha;
    s = s + (1.f - alpha) * gi * gi;
    so = s;
    po = pi - lr * gi / (sqrtf(s) + eps);
  };
  if (vec) {
    // float4 per thread (the flat buffers are 16-byte aligned), the n % 4
    // tail by the first threads; the same operations per element
    const int n4 = (int)(n / 4);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
      const float4 gv = reinterpret_cast<const float4*>(g)[i];
      const float4 sv = reinterpret_cast<const float4*>(sa)[i];
      const float4 pv = reinterpret_cast<const float4*>(p)[i];
      float4 po, so;
      upd(pv.x, gv.x, sv.x, po.x, so.x);
      upd(pv.y, gv.y, sv.y, po.y, so.y);
      upd(pv.z, gv.z, sv.z, po.z, so.z);
      upd(pv.w, gv.w, sv.w, po.w, so.w);
      reinterpret_cast<float4*>(sa)[i] = so;
      reinterpret_cast<float4*>(p)[i] = po;
    }
    const long long t = 4ll * n4 + blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (t < n) upd(p[t], g[t], sa[t], p[t], sa[t]);
    return;
  }
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    upd(p[i], g[i], sa[i], p[i], sa[i]);
}

template <typename T>
__global__ void adam_k(T* __restrict__ p, const T* __restrict__ g, T* __restrict__ m, T* __restrict__ v, long long n,
                       T lr, T b1, T b2, T eps, T bc1, T bc2sqrt) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const T gi = g[i];
    const T mi = m[i] * b1 + (T(1) - b1) * gi;
    const T vi = v[i] * b2 + (T(1) - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const T denom = sqrt(vi) / bc2sqrt + eps;
    p[i] = p[i] - (lr / bc1) * mi / denom;
  }
}

template <typename T>
__global__ void sgd_k(T* __restrict__ p, const T* __restrict__ g, T* __restrict__ buf, long long n, T lr, T mom,
                      int first) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    T d = g[i];
    if (buf) {
      const T b = first ? d : buf[i] * mom + d;
      buf[i] = b;
      d = b;
    }
    p[i] = p[i] - lr * d;
  }
}

static inline int grid_for(long long n) {
  long long g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

extern "C" {

const char* paig_last_error(void) { return g_err; }

// 2: paig_decoder_bwd(_blocks) take `live`; the paig_conv_wprep image starts
// with the channel-exponent header (round 3)
int paig_abi_version(void) { return PAIG_ABI_VERSION; }

// f16 range guard (common.h): waits for the device, then reads (and with
// clear != 0 resets) the flags the split-precision kernels set when an
// unscaled f16 operand reached |v| >= 65504.  1 = flagged, 0 = clean.
int paig_f16_range_status(int clear) {
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    paig_set_error("paig_f16_range_status: %s", hipGetErrorString(e));
    return -(int)e;
  }
  const int a = paig_f16_range_conv(clear), b = paig_f16_range_gemm(clear), c = paig_f16_range_bwd(clear);
  if (a < 0 || b < 0 || c < 0) {
    paig_set_error("paig_f16_range_status: flag read failed");
    return -1;
  }
  return (a | b | c) ? 1 : 0;
}

// y[P] = W2 tanh(W1 1 + b1) + b2 ; hout[200] ; ypost = sigmoid(y) if non-null
int paig_vfn_fwd_multi(int n, const float* const* W1, const float* const* b1, const float* const* W2,
                       const float* const* b2, float* const* hout, float* const* y, float* const* ypost, const int* P,
                       void* stream) {
  PAIG_REQUIRE(n >= 1 && n <= VMAX, "paig_vfn_fwd_multi: n=%d (1..%d)", n, VMAX);
  VfnFwdTasks T;
  vfn_fwd_tasks(T, n, W1, b1, W2, b2, hout, y, ypost, P);
  hipLaunchKernelGGL(vfn_fwd_k, dim3(T.blk0[n]), dim3(256), 0, (hipStream_t)stream, T);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_vfn_fwd(const float* W1, const float* b1, const float* W2, const float* b2, float* hout, float* y,
                 float* ypost, int P, void* stream) {
  return paig_vfn_fwd_multi(1, &W1, &b1, &W2, &b2, &hout, &y, &ypost, &P, stream);
}

int paig_vfn_bwd_blocks(int P) { return cdiv(P, VROWS); }

// d: adjoint of y (sig = 0) or of sigmoid(y) (sig = 1). part[k]: >= blocks(P[k])*200 floats.
static int vfn_bwd_launch(int n, const float* const* d, const float* const* y, const int* sig, const float* const* h,
                          const float* const* W2, float* const* dW1, float* const* db1, float* const* dW2,
                          float* const* db2, float* const* part, const int* P, void* stream, bool phase1_only) {
  PAIG_REQUIRE(n >= 1 && n <= VMAX, "paig_vfn_bwd_multi: n=%d (1..%d)", n, VMAX);
  VfnBwdTasks T;
  vfn_bwd_tasks(T, n, d, y, sig, h, W2, dW1, db1, dW2, db2, part, P);
  hipLaunchKernelGGL(vfn_bwd1_k, dim3(T.blk0[n]), dim3(256), 0, (hipStream_t)stream, T);
  PAIG_CHECK_LAUNCH();
  if (phase1_only) return 0;
  hipLaunchKernelGGL(vfn_bwd2_k, dim3(VH * n), dim3(64), 0, (hipStream_t)stream, T);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_vfn_bwd_multi(int n, const float* const* d, const float* const* y, const int* sig, const float* const* h,
                       const float* const* W2, float* const* dW1, float* const* db1, float* const* dW2,
                       float* const* db2, float* const* part, const int* P, void* stream) {
  return vfn_bwd_launch(n, d, y, sig, h, W2, dW1, db1, dW2, db2, part, P, stream, false);
}

// phase 1 only (dW2, db2 and the per-block partials of dh): phase 2 then runs
// inside paig_head_bwd_vel_vfn2's launch
int paig_vfn_bwd1_multi(int n, const float* const* d, const float* const* y, const int* sig, const float* const* h,
                        const float* const* W2, float* const* dW1, float* const* db1, float* const* dW2,
                        float* const* db2, float* const* part, const int* P, void* stream) {
  return vfn_bwd_launch(n, d, y, sig, h, W2, dW1, db1, dW2, db2, part, P, stream, true);
}

int paig_vfn_bwd(const float* d, const float* y, int sig, const float* h, const float* W2, float* dW1, float* db1,
                 float* dW2, float* db2, float* part, int P, void* stream) {
  return paig_vfn_bwd_multi(1, &d, &y, &sig, &h, &W2, &dW1, &db1, &dW2, &db2, &part, &P, stream);
}

int paig_loss_reduce(const float* sse_rec, const float* sse_roll, int B, int Te, int R, int pred, float ae, float* pred_out,
                     float* extrap_out, float* recons_out, void* stream) {
  hipLaunchKernelGGL(loss_reduce_k, dim3(1), dim3(1024), 0, (hipStream_t)stream, sse_rec, sse_roll, B, Te, R, pred,
                     ae, pred_out, extrap_out, recons_out);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_loss_bwd(const float* dpred, const float* dext, const float* drec, float ae, float* wrec, float* wroll, int B,
                  int Te, int R, int pred, void* stream) {
  hipLaunchKernelGGL(loss_bwd_k, dim3(grid_for((long long)B * (R > Te ? R : Te))), dim3(256), 0, (hipStream_t)stream,
                     dpred, dext, drec, ae, wrec, wroll, B, Te, R, pred);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_frame_sse(const float* a, long long a_fs, int a_grp, long long a_gs, const float* b, long long b_fs, int b_grp,
                   long long b_gs, float* sse, int F, int n, void* stream) {
  if (F <= 0) return 0;
  int g = F < 2048 ? F : 2048;
  hipLaunchKernelGGL(frame_sse_k, dim3(g), dim3(256), 0, (hipStream_t)stream, FView{a, a_fs, a_gs, a_grp},
                     FView{b, b_fs, b_gs, b_grp}, sse, F, n);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_frame_sse_bwd(const float* a, long long a_fs, int a_grp, long long a_gs, const float* b, long long b_fs,
                       int b_grp, long long b_gs, const float* w, float* da, int F, int n, void* stream) {
  if (F <= 0) return 0;
  hipLaunchKernelGGL(frame_sse_bwd_k, dim3(grid_for((long long)F * n)), dim3(256), 0, (hipStream_t)stream,
                     FView{a, a_fs, a_gs, a_grp}, FView{b, b_fs, b_gs, b_grp}, w, da, F, n);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_rmsprop_f32(float* p, const float* g, float* sa, long long n, float lr, float alpha, float eps, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(rmsprop_k<float>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, g, sa, n, lr, alpha, eps);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_rmsprop_mixed(float* p32, const float* g32, float* s32, long long n32, double* p64, const double* g64,
                       double* s64, long long n64, double lr, double alpha, double eps, void* stream) {
  if (n32 <= 0 && n64 <= 0) return 0;
  const int vec = n32 < (1ll << 31) && ((uintptr_t)p32 | (uintptr_t)g32 | (uintptr_t)s32) % 16 == 0;
  const long long nb = n32 > 0 ? (vec ? n32 / 4 + 1 : n32) : 1;
  hipLaunchKernelGGL(rmsprop_mixed_k, dim3(grid_for(nb)), dim3(256), 0, (hipStream_t)stream, p32, g32, s32, n32,
                     (float)lr, (float)alpha, (float)eps, p64, g64, s64, n64, lr, alpha, eps, vec);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_rmsprop_f64(double* p, const double* g, double* sa, long long n, double lr, double alpha, double eps,
                     void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(rmsprop_k<double>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, g, sa, n, lr, alpha,
                     eps);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_adam_f32(float* p, const float* g, float* m, float* v, long long n, float lr, float b1, float b2, float eps,
                  float bc1, float bc2sqrt, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(adam_k<float>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, lr, b1, b2,
                     eps, bc1, bc2sqrt);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_adam_f64(double* p, const double* g, double* m, double* v, long long n, double lr, double b1, double b2,
                  double eps, double bc1, double bc2sqrt, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(adam_k<double>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, lr, b1, b2,
                     eps, bc1, bc2sqrt);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_sgd_f32(float* p, const float* g, float* buf, long long n, float lr, float mom, int first, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(sgd_k<float>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, g, buf, n, lr, mom, first);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_sgd_f64(double* p, const double* g, double* buf, long long n, double lr, double mom, int first, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(sgd_k<double>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, g, buf, n, lr, mom, first);
  PAIG_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"

// d *= (y > 0): the ReLU derivative applied to a gradient in place (the
// standalone ShallowUNet backward: its last conv's output is ReLU'd, Q13)
__global__ void relu_mask_k(const float* __restrict__ y, float* __restrict__ d, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    d[i] = y[i] > 0.f ? d[i] : 0.f;
}

extern "C" {

int paig_relu_mask(const float* y, float* d, long long n, void* stream) {
  if (n <= 0) return 0;
  const int g = (int)(n / 256 + 1 < 4096 ? n / 256 + 1 : 4096);
  hipLaunchKernelGGL(relu_mask_k, dim3(g), dim3(256), 0, (hipStream_t)stream, y, d, n);
  PAIG_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
