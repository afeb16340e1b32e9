// VariableFromNetwork (nn/network/blocks.py:311-322) device code shared by
// the launches that run it: its own (misc.hip) and the velocity encoder's
// forward, which takes the VFN forward blocks into its grid (velmlp.hip: the
// two are independent, so one launch instead of two on the step's stream).
#pragma once
#include "common.h"

namespace paig_vfn {

constexpr int VH = 200;  // VariableFromNetwork hidden width (blocks.py:314)
constexpr int VIN = 10;  // ones[1, 10]

// The three VariableFromNetwork instances (template, content, background) of a
// step run as ONE launch per phase: a block finds its instance in a small
// task table (block ranges), so the three latency-bound GEMVs overlap.
constexpr int VMAX = 4;
struct VfnFwdTasks {
  const float* W1[VMAX];
  const float* b1[VMAX];
  const float* W2[VMAX];
  const float* b2[VMAX];
  float* hout[VMAX];
  float* y[VMAX];
  float* ypost[VMAX];
  int P[VMAX];
  int blk0[VMAX + 1];
  int n;
};
struct VfnBwdTasks {
  const float* d[VMAX];
  const float* y[VMAX];
  const float* h[VMAX];
  const float* W2[VMAX];
  float* dW1[VMAX];
  float* db1[VMAX];
  float* dW2[VMAX];
  float* db2[VMAX];
  float* part[VMAX];
  int sig[VMAX];
  int P[VMAX];
  int blk0[VMAX + 1];   // bwd1 block ranges (rows per block = VROWS)
  int n;
};
constexpr int VROWS = 8;

__device__ __forceinline__ int task_of(const int* blk0, int n, int b) {
  int k = 0;
  while (k + 1 < n && b >= blk0[k + 1]) ++k;
  return k;
}

// h = tanh(W1 @ ones + b1) in LDS; one wave per output row afterwards.
// (a block of 256 threads; blk = its index among the VFN blocks of the launch)
__device__ __forceinline__ void vfn_fwd_block(const VfnFwdTasks& T, int blk) {
  const int k = task_of(T.blk0, T.n, blk);
  const int bid = blk - T.blk0[k], nb = T.blk0[k + 1] - T.blk0[k];
  const float* __restrict__ W1 = T.W1[k];
  const float* __restrict__ W2 = T.W2[k];
  const int P = T.P[k];
  __shared__ float h[VH];
  for (int j = threadIdx.x; j < VH; j += blockDim.x) {
    float s = 0.f;
    for (int i = 0; i < VIN; ++i) s += W1[j * VIN + i];  // x = ones
    const float v = tanhf(s + T.b1[k][j]);
    h[j] = v;
    if (bid == 0) T.hout[k][j] = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wg = (bid * blockDim.x + threadIdx.x) >> 6;
  const int nw = (nb * blockDim.x) >> 6;
  for (int p = wg; p < P; p += nw) {
    float s = 0.f;
    for (int j = lane; j < VH; j += 64) s = fmaf(W2[(long long)p * VH + j], h[j], s);
    s = wave_sum(s);
    if (lane == 0) {
      const float v = s + T.b2[k][p];
      T.y[k][p] = v;
      if (T.ypost[k]) T.ypost[k][p] = 1.f / (1.f + expf(-v));
    }
  }
}


// the forward task table of n <= VMAX instances; returns its block count
inline int vfn_fwd_tasks(VfnFwdTasks& T, int n, const float* const* W1, const float* const* b1,
                         const float* const* W2, const float* const* b2, float* const* hout, float* const* y,
                         float* const* ypost, const int* P) {
  T = VfnFwdTasks{};
  T.n = n;
  T.blk0[0] = 0;
  for (int k = 0; k < n; ++k) {
    T.W1[k] = W1[k];
    T.b1[k] = b1[k];
    T.W2[k] = W2[k];
    T.b2[k] = b2[k];
    T.hout[k] = hout[k];
    T.y[k] = y[k];
    T.ypost[k] = ypost ? ypost[k] : nullptr;
    T.P[k] = P[k];
    int g = (P[k] + 3) / 4;
    if (g > 1024) g = 1024;
    if (g < 1) g = 1;
    T.blk0[k + 1] = T.blk0[k] + g;
  }
  return T.blk0[n];
}

// backward phase 2, one item = (instance k, hidden unit j) on one 64-lane
// wave: dh[j] = the phase-1 block partials summed, the tanh', and the first
// layer's grads (input = ones)
__device__ __forceinline__ void vfn_bwd2_item(const VfnBwdTasks& T, int item, int lane) {
  const int k = item / VH, j = item % VH;
  const int nblk = T.blk0[k + 1] - T.blk0[k];
  const float* __restrict__ part = T.part[k];
  float s = 0.f;
  for (int b = lane; b < nblk; b += 64) s += part[b * VH + j];
  s = wave_sum(s);
  const float hj = T.h[k][j];
  const float g = s * (1.f - hj * hj);
  if (lane < VIN) T.dW1[k][j * VIN + lane] = g;
  if (lane == 0) T.db1[k][j] = g;
}

// the backward task table of n <= VMAX instances; returns phase 1's block count
inline int vfn_bwd_tasks(VfnBwdTasks& T, int n, const float* const* d, const float* const* y, const int* sig,
                         const float* const* h, const float* const* W2, float* const* dW1, float* const* db1,
                         float* const* dW2, float* const* db2, float* const* part, const int* P) {
  T = VfnBwdTasks{};
  T.n = n;
  T.blk0[0] = 0;
  for (int k = 0; k < n; ++k) {
    T.d[k] = d[k];
    T.y[k] = y[k];
    T.sig[k] = sig[k];
    T.h[k] = h[k];
    T.W2[k] = W2[k];
    T.dW1[k] = dW1[k];
    T.db1[k] = db1[k];
    T.dW2[k] = dW2[k];
    T.db2[k] = db2[k];
    T.part[k] = part[k];
    T.P[k] = P[k];
    T.blk0[k + 1] = T.blk0[k] + (P[k] + VROWS - 1) / VROWS;
  }
  return T.blk0[n];
}

}  // namespace paig_vfn
