// Shared device helpers of the split-precision MFMA convolutions
// (conv_split.hip: forward / dgrad / wgrad; conv_bwd.hip: the fused layer
// backward): 16-bit fragment types, the hi/lo split, the three-MFMA product,
// transposed LDS reads, XCD-aware tile order and the fused 2x upsample stage.
#pragma once
#include "conv_tile.h"

#ifndef PAIG_SCALE_MODE
#define PAIG_SCALE_MODE 0   // A/B experiments only: 1 no weight scale, 2 no scaling
#endif

namespace {

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr int rup(int a, int b) { return ceil_div(a, b) * b; }

// Physical tile of persistent-loop tile L.  Workgroups sit on XCD
// (id mod 8), each XCD with its own L2; with the grid a multiple of 8, the
// tiles of one XCD are L = x, x + 8, ...  Renumbering them into one
// contiguous run keeps neighbouring row blocks of a frame (which re-read
// each other's halo rows) on one XCD, processed at the same time.
__device__ __forceinline__ int xcd_tile(int L, int ntiles) {
  return (ntiles % 8 == 0 && gridDim.x % 8 == 0) ? (L % 8) * (ntiles / 8) + L / 8 : L;
}
// largest divisor d of n with d * w <= cap (at least 1): rows per tile
constexpr int rows_fit(int n, int w, int cap) {
  int best = 1;
  for (int d = 1; d <= n; ++d)
    if (n % d == 0 && d * w <= cap) best = d;
  return best;
}
// smallest y >= x with y % 16 == r
constexpr int to_mod16(int x, int r) { return x + ((r - x % 16) + 16) % 16; }

// rmax: running max |v| of the f16-split values (the range guard, common.h)
template <int PM>
__device__ __forceinline__ void split(float v, short& h, short& l, float& rmax) {
  if constexpr (PM == 0) {
    rmax = fmaxf(rmax, fabsf(v));
    const _Float16 a = (_Float16)v;
    const _Float16 b = (_Float16)(v - (float)a);
    h = __builtin_bit_cast(short, a);
    l = __builtin_bit_cast(short, b);
  } else {
    const __bf16 a = (__bf16)v;
    h = __builtin_bit_cast(short, a);
    if constexpr (PM == 1) {
      const __bf16 b = (__bf16)(v - (float)a);
      l = __builtin_bit_cast(short, b);
    } else {
      l = 0;
    }
  }
}

template <int PM>
__device__ __forceinline__ f32x4 mma(s16x8 a, s16x8 b, f32x4 c) {
  if constexpr (PM == 0)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                  0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
}

// acc += a*b with both operands split (hi, lo); PM 2 uses the hi parts only
template <int PM>
__device__ __forceinline__ f32x4 mma3(s16x8 ah, s16x8 al, s16x8 bh, s16x8 bl, f32x4 c) {
  if constexpr (PM != 2) {
    c = mma<PM>(al, bh, c);
    c = mma<PM>(ah, bl, c);
  }
  return mma<PM>(ah, bh, c);
}

__device__ __forceinline__ s16x4 tr_read(const short* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p);
}

// Fused 2x bilinear upsample input (c7, c10: the reference's torchvision
// Resize feeding a conv, blocks.py:260,269): a tile's half-resolution source
// window (rows y0/2 - 1 .. y0/2 + RT/2, all columns, fp32) is prefetched a
// tile ahead into registers, parked in LDS, and the upsampled rows are formed
// from LDS while building the 16-bit operand image.
#ifndef PAIG_UPS_CPAD
#define PAIG_UPS_CPAD 0   // A/B builds: floats of padding after each channel's window rows (4 measured neutral)
#endif
// the window's LDS floats: each channel's rows, then PAIG_UPS_CPAD floats
// (16 B of padding moves the interpolation's reads of channels 4 apart onto
// other banks; whole-step A/B: no change on spring / 3bp / mnist)
constexpr int up_pitch(int RT, int W) { return (RT / 2 + 2 + (RT & 1)) * (W / 2) + PAIG_UPS_CPAD; }
constexpr int up_window_floats(int CIN, int FPT, int RT, int W) { return FPT * CIN * up_pitch(RT, W); }

template <int CIN, int H, int W, int FPT, int RT>
struct UpStage {
  // window rows y0/2 - 1 .. : RT/2 + 2 rows for an even tile height, one more
  // for an odd one (3bp's 18-row frames tile as 2 x 9 rows)
  static constexpr int HS = H / 2, WS = W / 2, SRN = RT / 2 + 2 + (RT & 1);
  static constexpr int VS = WS % 4 == 0 ? 4 : 1;               // floats per load unit
  static constexpr int QS = WS / VS;
  static constexpr int NSU = FPT * CIN * SRN * QS, NLS = (NSU + 255) / 256;
  static constexpr int CP = up_pitch(RT, W);         // floats per (frame, channel)
  static constexpr int SL = up_window_floats(CIN, FPT, RT, W);   // floats of LDS
  f32x4 v[VS == 4 ? NLS : 1];
  float v1[VS == 1 ? NLS : 1];
  __device__ __forceinline__ void issue(const FView& x, int F, int f0, int y0, int tid) {
#pragma unroll
    for (int l = 0; l < NLS; ++l) {
      const int i = tid + l * 256;
      const int q = i % QS, sr = (i / QS) % SRN, c = (i / (QS * SRN)) % CIN, fi = i / (QS * SRN * CIN);
      const int srow = y0 / 2 - 1 + sr;
      const bool ok = i < NSU && f0 + fi < F && srow >= 0 && srow < HS;
      const float* src = ok ? x.frame(f0) + fi * (int)x.fs + c * HS * WS + srow * WS + VS * q : paig_zeros;
      if constexpr (VS == 4) v[l] = *reinterpret_cast<const f32x4*>(src);
      else v1[l] = *src;
    }
  }
  // max |v| of the prefetched window: a bound on its upsampled values (convex
  // combinations of window values)
  __device__ __forceinline__ float amax() const {
    float m = 0.f;
#pragma unroll
    for (int l = 0; l < NLS; ++l) {
      if constexpr (VS == 4) m = amax2(amax2(m, v[l][0], v[l][1]), v[l][2], v[l][3]);
      else m = fmaxf(m, fabsf(v1[l]));
    }
    return m;
  }
  __device__ __forceinline__ void commit(float* Sl, int tid) const {
#pragma unroll
    for (int l = 0; l < NLS; ++l) {
      const int i = tid + l * 256;   // Sl is [fi][c][CP]: rows sr of WS floats, then the padding
      if (NSU % 256 != 0 && i >= NSU) break;
      const int fc = i / (QS * SRN), r = i % (QS * SRN);
      if constexpr (VS == 4) *reinterpret_cast<f32x4*>(Sl + fc * CP + 4 * r) = v[l];
      else Sl[fc * CP + r] = v1[l];
    }
  }
  // output pixel (row gy, column x) of channel c of frame fi (0 <= gy < H), in
  // aten's upsample_bilinear2d operation order
  static __device__ __forceinline__ float px1(const float* Sl, int fi, int c, int gy, int y0, int x) {
    int ya, yb, xa, xb;
    float wa, wb, ua, ub;
    up2_taps(gy, HS, ya, yb, wa, wb);
    up2_taps(x, WS, xa, xb, ua, ub);
    const float* p = Sl + (fi * CIN + c) * CP;
    const float* r0 = p + (ya - (y0 / 2 - 1)) * WS;
    const float* r1 = p + (yb - (y0 / 2 - 1)) * WS;
    return wa * (ua * r0[xa] + ub * r0[xb]) + wb * (ua * r1[xa] + ub * r1[xb]);
  }
  // output pixels (row gy, x = 4q..4q+3) of channel c of frame fi (0 <= gy < H)
  static __device__ __forceinline__ f32x4 row4(const float* Sl, int fi, int c, int gy, int y0, int q) {
    int ya, yb;
    float wa, wb;
    up2_taps(gy, HS, ya, yb, wa, wb);
    const float* p = Sl + (fi * CIN + c) * CP;
    const float* r0 = p + (ya - (y0 / 2 - 1)) * WS;
    const float* r1 = p + (yb - (y0 / 2 - 1)) * WS;
    const int c0 = q > 0 ? 2 * q - 1 : 0, c3 = 2 * q + 2 < WS ? 2 * q + 2 : WS - 1;
    const float2 m0 = *reinterpret_cast<const float2*>(r0 + 2 * q);
    const float2 m1 = *reinterpret_cast<const float2*>(r1 + 2 * q);
    const float a0 = r0[c0], a3 = r0[c3], b0 = r1[c0], b3 = r1[c3];
    const float w0 = q > 0 ? 0.25f : 0.f, w1 = q > 0 ? 0.75f : 1.f;
    f32x4 o;
    o[0] = wa * (w0 * a0 + w1 * m0.x) + wb * (w0 * b0 + w1 * m1.x);
    o[1] = wa * (0.75f * m0.x + 0.25f * m0.y) + wb * (0.75f * m1.x + 0.25f * m1.y);
    o[2] = wa * (0.25f * m0.x + 0.75f * m0.y) + wb * (0.25f * m1.x + 0.75f * m1.y);
    o[3] = wa * (0.75f * m0.y + 0.25f * a3) + wb * (0.75f * m1.y + 0.25f * b3);
    return o;
  }
  // output rows gy (odd) and gy + 1 at once (pixels 4q..4q+3): 2x bilinear
  // output rows 2k+1 and 2k+2 interpolate the same source rows k, k+1, so the
  // row reads and the horizontal interpolations are shared; each row's
  // vertical weights are its own (row4's operation order).  ok0 / ok1: the
  // rows lie in the frame (else 0; the taps then come from the valid row)
  static __device__ __forceinline__ void row4x2(const float* Sl, int fi, int c, int gy, int y0, int q, bool ok0,
                                                bool ok1, f32x4& o0, f32x4& o1) {
    int ya, yb, ya1, yb1;
    float wa0, wb0, wa1, wb1;
    up2_taps(gy, HS, ya, yb, wa0, wb0);
    up2_taps(gy + 1, HS, ya1, yb1, wa1, wb1);
    if (!ok0) {
      ya = ya1;
      yb = yb1;
    }
    const float* p = Sl + (fi * CIN + c) * CP;
    const float* r0 = p + (ya - (y0 / 2 - 1)) * WS;
    const float* r1 = p + (yb - (y0 / 2 - 1)) * WS;
    const int c0 = q > 0 ? 2 * q - 1 : 0, c3 = 2 * q + 2 < WS ? 2 * q + 2 : WS - 1;
    const float2 m0 = *reinterpret_cast<const float2*>(r0 + 2 * q);
    const float2 m1 = *reinterpret_cast<const float2*>(r1 + 2 * q);
    const float a0 = r0[c0], a3 = r0[c3], b0 = r1[c0], b3 = r1[c3];
    const float w0 = q > 0 ? 0.25f : 0.f, w1 = q > 0 ? 0.75f : 1.f;
    const float h0[4] = {w0 * a0 + w1 * m0.x, 0.75f * m0.x + 0.25f * m0.y, 0.25f * m0.x + 0.75f * m0.y,
                         0.75f * m0.y + 0.25f * a3};
    const float h1[4] = {w0 * b0 + w1 * m1.x, 0.75f * m1.x + 0.25f * m1.y, 0.25f * m1.x + 0.75f * m1.y,
                         0.75f * m1.y + 0.25f * b3};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o0[j] = ok0 ? wa0 * h0[j] + wb0 * h1[j] : 0.f;
      o1[j] = ok1 ? wa1 * h0[j] + wb1 * h1[j] : 0.f;
    }
  }
};

// LDS available to one block (gfx950: 160 KB per CU)
constexpr int LDS_MAX = 160 * 1024;

}  // namespace
