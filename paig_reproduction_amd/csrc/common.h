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

// the declarations every entry point must match (and PAIG_ABI_VERSION)
#include "../../include/paig_hip.h"

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

// v / 255 correctly rounded (= IEEE division, as numpy) for v in 0..255:
// the reciprocal product plus one fma correction of its exact residual
// (checked for all 256 values by tests/test_device_data.py).  The batch
// gather and the decoders' uint8 targets both use it, so a target read from
// the bytes equals the gathered fp32 value bit for bit.
__device__ __forceinline__ float div255(float v) {
  constexpr float r = 1.0f / 255.0f;
  const float q = v * r;
  return __builtin_fmaf(__builtin_fmaf(-q, 255.0f, v), r, q);
}

// The loss weight (dL/dSSE) of frame f from the loss adjoints
// (physics_models.py:119-142; quirk Q2: dt is the adjoint of train = pred +
// ae * recons): mode 2 rollout frames (step f % R; the first pred steps carry
// dt / (B pred), the others de / (B (R - pred))), mode 1 reconstruction
// frames ((ae dt + dr) / (B Te)).  Adjoints may be null (= 0).  paig_loss_bwd
// writes these values and the decoder backwards form them in-kernel: one
// function, so both give the same bits.
__device__ __forceinline__ float loss_weight(int mode, int f, const float* dt, const float* de, const float* dr,
                                             float ae, int B, int Te, int R, int pred) {
  const float t = dt ? *dt : 0.f;
  if (mode == 2) return (f % R) < pred ? t / (float)(B * pred) : ((de && R > pred) ? *de / (float)(B * (R - pred)) : 0.f);
  const float d = (ae > 0.f ? ae * t : 0.f) + (dr ? *dr : 0.f);
  return d / (float)(B * Te);
}

struct FViewW {
  float* p;
  long long fs;
  __device__ __forceinline__ float* frame(int f) const { return p + (long long)f * fs; }
};

// The fused 2x2 max pool's outputs of a forward conv (flags & 64): the pooled
// frames and, optionally, one window code byte per (channel, pooled pixel):
// bits 0-3 the ReLU' mask (value > 0) of the window's pixels (y, x),
// (y, x+1), (y+1, x), (y+1, x+1); bits 4-5 the argmax among them in aten's
// max_pool2d scan order.  Code layout per frame (code_fs bytes):
// [channel / 8][H/2][W/2][channel % 8] -- a consumer staging 8 channels of one
// window reads one 8-byte word.
struct PoolOut {
  float* p;
  long long fs;
  unsigned char* code;
  long long code_fs;
  __device__ __forceinline__ float* frame(int f) const { return p + (long long)f * fs; }
};

static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

__device__ __forceinline__ int uniform_i(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ float uniform_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
}

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

// f16 range guard of the split-precision kernels (conv_split.hip, gemm.hip):
// their unscaled f16 operands (activations, weights) need |v| < 65504.  A
// kernel that stages a larger value sets its translation unit's flag (plain
// vector store; any value, so concurrent writers need no atomics);
// paig_f16_range_status() reads and clears every unit's flag.
static __device__ unsigned paig_f16_range_flag;
constexpr float PAIG_F16_MAX = 65504.f;
__device__ __forceinline__ void f16_range_note(float rmax) {
  if (rmax >= PAIG_F16_MAX) *(volatile unsigned*)&paig_f16_range_flag = 1u;
}
// host side: read (and clear) this unit's flag; the device must be idle
#define PAIG_F16_RANGE_ACCESSOR(NAME)                                                     \
  int NAME(int clear) {                                                                   \
    unsigned v = 0;                                                                       \
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(paig_f16_range_flag), sizeof(v)) != hipSuccess) \
      return -1;                                                                          \
    if (clear && v) {                                                                     \
      const unsigned z = 0;                                                               \
      if (hipMemcpyToSymbol(HIP_SYMBOL(paig_f16_range_flag), &z, sizeof(z)) != hipSuccess) \
        return -1;                                                                        \
    }                                                                                     \
    return (int)v;                                                                        \
  }
int paig_f16_range_conv(int clear);
int paig_f16_range_gemm(int clear);
int paig_f16_range_bwd(int clear);

// fixed power-of-two scale of the fallback paths (a conv weight gradient
// without the forward's recorded X maximum, GEMM math 4 / 5's fixed operand):
// full f16 precision for |v| >= 2^-11, a range-flagged overflow at 2^8.  The
// training step scales every operand dynamically (per tile, per output
// channel, running per block) instead.
#define PAIG_A_EXP 8

// power-of-two exponent e with m * 2^e in [2^14, 2^15) (f16's top binade,
// clear of its 65504 limit); 100 when m == 0 (no constraint); clamped
// m must be wave-uniform (a block maximum); the exponent is computed in
// scalar registers
__device__ __forceinline__ int f16_scale_exp(float m) {
  const int b = __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, m));
  int e = b > 0 ? 14 - (((b >> 23) & 255) - 127) : 100;
  return e < -100 ? -100 : (e > 100 ? 100 : e);
}

// per-lane form of f16_scale_exp (m >= 0 need not be uniform; 0 for m == 0)
__device__ __forceinline__ int f16_scale_exp_v(float m) {
  const int b = __builtin_bit_cast(int, m);
  int e = b > 0 ? 14 - (((b >> 23) & 255) - 127) : 0;
  return e < -100 ? -100 : (e > 100 ? 100 : e);
}

// max over the wave of v >= 0, returned wave-uniform: DPP within rows of 16
// (quad swaps, half-row and row mirrors: VALU ops, no LDS round trips), then
// the four row results read as scalars.  Non-negative floats order as their
// bit patterns, so the steps are integer maxima (no NaN canonicalisation).
// The scale exponents of the split-precision kernels need it once per tile.
template <int CTRL>
__device__ __forceinline__ unsigned dpp_umax(unsigned v) {
  const unsigned o = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
  return v > o ? v : o;
}
__device__ __forceinline__ float wave_max_u(float f) {
  unsigned v = __builtin_bit_cast(unsigned, f);
  v = dpp_umax<0xB1>(v);    // quad_perm [1,0,3,2]
  v = dpp_umax<0x4E>(v);    // quad_perm [2,3,0,1]
  v = dpp_umax<0x141>(v);   // row_half_mirror: quads 0<->1, 2<->3
  v = dpp_umax<0x140>(v);   // row_mirror: halves of the row
  const unsigned r0 = __builtin_amdgcn_readlane((int)v, 0), r1 = __builtin_amdgcn_readlane((int)v, 16);
  const unsigned r2 = __builtin_amdgcn_readlane((int)v, 32), r3 = __builtin_amdgcn_readlane((int)v, 48);
  const unsigned a = r0 > r1 ? r0 : r1, b = r2 > r3 ? r2 : r3;
  return __builtin_bit_cast(float, a > b ? a : b);
}

// Source of the zeros a branch-free staging load reads for an out-of-range
// element: selecting the ADDRESS (instead of the loaded data) keeps the load
// unconsumed until its use, so a prefetch really stays in flight behind the
// MFMAs; a data select made the compiler wait for it right after issue.
static __device__ __attribute__((aligned(16))) float paig_zeros[4];   // never written
// zero planes for staging units that read several channel planes from one
// base address (8 channels of up to 64 x 64 pixels, + one float2 beyond)
static __device__ __attribute__((aligned(16))) float paig_zero_planes[8 * 4096 + 4];

// f16 hi + lo pieces of two fp32 values already scaled into f16's range,
// each pair packed (a in the low half): one packed RNE conversion per piece
// and a packed residual, ~3 VALU ops per value
typedef float pf32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 pf16x2 __attribute__((ext_vector_type(2)));
struct HiLo {
  unsigned h, l;
};
__device__ __forceinline__ HiLo split_pk(float a, float b) {
  const pf32x2 v = {a, b};
  const pf16x2 hh = __builtin_convertvector(v, pf16x2);
  const pf16x2 ll = __builtin_convertvector(v - __builtin_convertvector(hh, pf32x2), pf16x2);
  return HiLo{__builtin_bit_cast(unsigned, hh), __builtin_bit_cast(unsigned, ll)};
}
// m = max(m, |a|, |b|): one v_max3 with abs modifiers (m stays canonical)
__device__ __forceinline__ float amax2(float m, float a, float b) { return fmaxf(fmaxf(m, fabsf(a)), fabsf(b)); }

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// fp64 wave sum without LDS round trips (the __shfl_xor form above issues two
// ds_bpermute per step): DPP within rows of 16 (quad swaps, half-row and row
// mirrors; a + b and b + a round alike, so every lane of a row holds the same
// row sum), then the four row sums read as scalars and added in a fixed
// order.  Returned wave-uniform; deterministic.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  // every lane reads a valid source lane in these patterns: bound_ctrl, no
  // "old" operand to initialise
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)b, CTRL, 0xF, 0xF, true);
  const unsigned hi = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)(b >> 32), CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, (unsigned long long)lo | ((unsigned long long)hi << 32));
}
// N independent fp64 sums within each row of 16 lanes, the DPP stages
// interleaved across the N values (ILP): afterwards every lane of a row holds
// that row's sums
template <int N>
__device__ __forceinline__ void row_sums_dpp_d(double* v) {
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += dpp_d<0xB1>(v[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += dpp_d<0x4E>(v[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += dpp_d<0x141>(v[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += dpp_d<0x140>(v[i]);
}
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
// fp32 wave sum through DPP row reductions + 4 readlanes (wave-uniform result)
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  v += dpp_f<0x140>(v);
  const auto rl = [&](int l) { return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l)); };
  return (rl(0) + rl(16)) + (rl(32) + rl(48));
}
__device__ __forceinline__ double readlane_d(double v, int l) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
  return __builtin_bit_cast(double, (unsigned long long)lo | ((unsigned long long)hi << 32));
}
__device__ __forceinline__ double wave_sum_dpp_d(double v) {
  v += dpp_d<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_d<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_d<0x141>(v);   // row_half_mirror
  v += dpp_d<0x140>(v);   // row_mirror
  return (readlane_d(v, 0) + readlane_d(v, 16)) + (readlane_d(v, 32) + readlane_d(v, 48));
}

// GEMM epilogue (gemm.hip, dense.hip): activation of the output, then the
// derivative of a stored activation (aux) for a backward GEMM
enum { ACT_NONE = 0, ACT_RELU = 1, ACT_TANH = 2, ACT_SIGMOID = 3 };
enum { AUX_NONE = 0, AUX_RELU = 1, AUX_TANH = 2 };
__device__ __forceinline__ float epi(float v, int act, int auxm, const float* aux, long long aoff) {
  if (act == ACT_RELU) v = v < 0.f ? 0.f : v;
  else if (act == ACT_TANH) v = tanhf(v);
  else if (act == ACT_SIGMOID) v = 1.f / (1.f + expf(-v));
  if (auxm == AUX_RELU) v = aux[aoff] > 0.f ? v : 0.f;
  else if (auxm == AUX_TANH) { float t = aux[aoff]; v = v * (1.f - t * t); }
  return v;
}
void paig_gemm_splitk_finish(int M, int N, int S, const float* part, float* C, long long ldc, float beta,
                             const float* bias, int act, int auxm, const float* aux, long long ldaux,
                             const float* rowpart, float* rowsum, hipStream_t st);

// MFMA implicit-GEMM convolutions (conv_mfma.hip): return 1 when the shape is
// instantiated there (launch status in *rc), 0 to fall back to the VALU path.
// xmax (nullable): per-block max |input| of a split-precision forward
// (written, n slots) / of the wgrad's X (read: the launch's fixed X scale)
struct XMax {
  float* p;
  int n;
  float* z = nullptr;   // forward only: zn floats to zero (paig_conv_fwd_prezero)
  int zn = 0;
};
// The U-Net forward's max-|x| slots of the layers after the first are zeroed
// by the first split forward launch instead of a separate memset: set the
// range, launch; paig_conv_fwd_prezero_pending() then says (and clears)
// whether no split forward took it (the caller must zero the slots itself).
void paig_conv_fwd_prezero(float* z, int zn);
bool paig_conv_fwd_prezero_pending();
int paig_conv_mfma_fwd(FView in, FViewW out, FView aux, const float* w, const float* b, int F, int Cin, int Cout,
                       int H, int W, int ks, int flags, hipStream_t st, int* rc, XMax xm, const void* wp = nullptr,
                       PoolOut pout = PoolOut{nullptr, 0, nullptr, 0});
int paig_conv_mfma_wgrad(FView x, FView dy, float* slab, int nblk_max, int* nblk_out, int F, int Cin, int Cout, int H,
                         int W, int ks, int flags, hipStream_t st, int* rc, XMax xm);
// Split-precision 16-bit MFMA convolutions (conv_split.hip), selected by
// flags & 128 (f16x3 forward / bf16x3 dgrad and wgrad) or flags & 256 (bf16).
int paig_conv_split_fwd(FView in, FViewW out, FView aux, const float* w, const float* b, int F, int Cin, int Cout,
                        int H, int W, int ks, int flags, hipStream_t st, int* rc, XMax xm, const void* wp = nullptr,
                        PoolOut pout = PoolOut{nullptr, 0, nullptr, 0});
int paig_conv_split_wgrad(FView x, FView dy, float* slab, int nblk_max, int* nblk_out, int F, int Cin, int Cout,
                          int H, int W, int ks, int flags, hipStream_t st, int* rc, XMax xm,
                          PoolOut pin = PoolOut{nullptr, 0, nullptr, 0});
int paig_conv_split_supported(int what, int Cin, int Cout, int H, int W, int ks, int flags);
