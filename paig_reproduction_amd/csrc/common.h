// Shared helpers for the PhysicsNet HIP kernels (gfx950 / CDNA4).
//
// Conventions of the C ABI (include/paig_hip.h):
//   * every entry point returns 0 on success, a PAIG_E_* code or a hipError_t;
//     it never throws or aborts; paig_last_error() has the message.
//   * all tensors are device pointers, fp32 unless the name says f64;
//     frames are [F][C][H][W] with a per-frame stride ("frame views").
//   * the library never allocates: the caller (PyTorch's caching allocator)
//     owns every buffer, workspaces included; calls are async on `stream`.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PAIG_E_SHAPE 1001
#define PAIG_E_UNSUPPORTED 1002

extern "C" const char* paig_last_error(void);
void paig_set_error(const char* fmt, ...);

#define PAIG_CHECK_LAUNCH()                                                  \
  do {                                                                       \
    hipError_t _e = hipGetLastError();                                       \
    if (_e != hipSuccess) {                                                  \
      paig_set_error("%s: launch failed: %s", __func__, hipGetErrorString(_e)); \
      return (int)_e;                                                        \
    }                                                                        \
  } while (0)

#define PAIG_REQUIRE(cond, ...)          \
  do {                                   \
    if (!(cond)) {                       \
      paig_set_error(__VA_ARGS__);       \
      return PAIG_E_SHAPE;               \
    }                                    \
  } while (0)

// A frame view: frame f of a [.., C, H, W] activation lives at
//   p + (grp > 0 ? (f / grp) * fs + (f % grp) * gs : f * fs)
// grp > 0 addresses the first frames of each sequence of a [B, T, C, H, W]
// input in place (frames n = b * grp + t, t < grp), without a copy.
struct FView {
  const float* p;
  long long fs;
  long long gs;
  int grp;
  __device__ __forceinline__ const float* frame(int f) const {
    return grp > 0 ? p + (long long)(f / grp) * fs + (long long)(f % grp) * gs : p + (long long)f * fs;
  }
};

struct FViewW {
  float* p;
  long long fs;
  __device__ __forceinline__ float* frame(int f) const { return p + (long long)f * fs; }
};

static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

__device__ __forceinline__ int uniform_i(int v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// MFMA implicit-GEMM convolutions (conv_mfma.hip): return 1 when the shape is
// instantiated there (launch status in *rc), 0 to fall back to the VALU path.
int paig_conv_mfma_fwd(FView in, FViewW out, FView aux, const float* w, const float* b, int F, int Cin, int Cout,
                       int H, int W, int ks, int flags, hipStream_t st, int* rc);
int paig_conv_mfma_wgrad(FView x, FView dy, float* slab, int nblk_max, int* nblk_out, int F, int Cin, int Cout, int H,
                         int W, int ks, int flags, hipStream_t st, int* rc);
// Split-precision 16-bit MFMA convolutions (conv_split.hip), selected by
// flags & 128 (f16x3 forward / bf16x3 dgrad and wgrad) or flags & 256 (bf16).
int paig_conv_split_fwd(FView in, FViewW out, FView aux, const float* w, const float* b, int F, int Cin, int Cout,
                        int H, int W, int ks, int flags, hipStream_t st, int* rc);
int paig_conv_split_wgrad(FView x, FView dy, float* slab, int nblk_max, int* nblk_out, int F, int Cin, int Cout,
                          int H, int W, int ks, int flags, hipStream_t st, int* rc);
int paig_conv_split_supported(int what, int Cin, int Cout, int H, int W, int ks, int flags);
