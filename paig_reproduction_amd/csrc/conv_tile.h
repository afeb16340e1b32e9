// Shared tile helpers of the MFMA convolution kernels (conv_mfma.hip: exact
// fp32 MFMA; conv_split.hip: split-precision 16-bit MFMA).
#pragma once
#include "common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int ceil_div(int a, int b) { return (a + b - 1) / b; }
constexpr int pad16mod32(int x) { return ((x + 15) / 16 * 16) % 32 == 0 ? (x + 15) / 16 * 16 + 16 : (x + 15) / 16 * 16; }
// smallest y >= x with y % 32 == r
constexpr int to_mod32(int x, int r) { return x + ((r - x % 32) + 32) % 32; }

// aten upsample_bilinear2d taps for an exact 2x upscale (scale 0.5, align_corners=False)
__device__ __forceinline__ void up2_taps(int d, int n, int& i0, int& i1, float& l0, float& l1) {
  float s = 0.5f * ((float)d + 0.5f) - 0.5f;
  if (s < 0.f) s = 0.f;
  i0 = (int)s;
  if (i0 > n - 1) i0 = n - 1;
  i1 = i0 + (i0 < n - 1 ? 1 : 0);
  l1 = s - (float)i0;
  l0 = 1.f - l1;
}

// 4 consecutive pixels (row gy, x = 4q..4q+3) of a conv input plane of size
// H x W: read directly (UPS = false) or formed on the fly as the 2x bilinear
// upsample of a (H/2 x W/2) source plane (UPS = true: the reference's
// torchvision Resize feeding c7/c10, blocks.py:289-290,298-299, never
// materialised).
template <bool UPS, int H, int W>
__device__ __forceinline__ f32x4 load_row4(const float* __restrict__ plane, int gy, int q) {
  if (!UPS) return *reinterpret_cast<const f32x4*>(plane + (long long)gy * W + 4 * q);
  constexpr int HS = H / 2, WS = W / 2;
  int y0, y1;
  float wy0, wy1;
  up2_taps(gy, HS, y0, y1, wy0, wy1);
  // x = 4q..4q+3 read source columns 2q-1 .. 2q+2 (clamped): 4 loads per row;
  // the horizontal weights are the constants up2_taps yields for 2x
  const int c0 = q > 0 ? 2 * q - 1 : 0, c3 = 2 * q + 2 < WS ? 2 * q + 2 : WS - 1;
  const float* r0 = plane + y0 * WS;
  const float* r1 = plane + y1 * WS;
  const float2 m0 = *reinterpret_cast<const float2*>(r0 + 2 * q);
  const float2 m1 = *reinterpret_cast<const float2*>(r1 + 2 * q);
  const float a0 = r0[c0], a3 = r0[c3], b0 = r1[c0], b3 = r1[c3];
  const float w0 = q > 0 ? 0.25f : 0.f, w1 = q > 0 ? 0.75f : 1.f;
  f32x4 v;
  v[0] = wy0 * (w0 * a0 + w1 * m0.x) + wy1 * (w0 * b0 + w1 * m1.x);
  v[1] = wy0 * (0.75f * m0.x + 0.25f * m0.y) + wy1 * (0.75f * m1.x + 0.25f * m1.y);
  v[2] = wy0 * (0.25f * m0.x + 0.75f * m0.y) + wy1 * (0.25f * m1.x + 0.75f * m1.y);
  v[3] = wy0 * (0.75f * m0.y + 0.25f * a3) + wy1 * (0.75f * m1.y + 0.25f * b3);
  return v;
}

// The same 4-pixel row segment split in two halves for software pipelining:
// issue() only starts the global loads (into registers, for the NEXT tile or
// channel chunk), finish() -- after the current tile's MFMAs -- forms the
// values (the 2x interpolation when UPS).  Out-of-range segments are zeros.
template <bool UPS, int H, int W>
struct Seg {
  f32x4 v;
  __device__ __forceinline__ void issue(const float* __restrict__ plane, int gy, int q, bool ok) {
    v = ok ? *reinterpret_cast<const f32x4*>(plane + (long long)gy * W + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  __device__ __forceinline__ f32x4 finish(int, int) const { return v; }
};

template <int H, int W>
struct Seg<true, H, W> {
  static constexpr int HS = H / 2, WS = W / 2;
  float2 m0, m1;
  float a0, a3, b0, b3;
  __device__ __forceinline__ void issue(const float* __restrict__ plane, int gy, int q, bool ok) {
    if (!ok) {
      m0 = m1 = make_float2(0.f, 0.f);
      a0 = a3 = b0 = b3 = 0.f;
      return;
    }
    int y0, y1;
    float wy0, wy1;
    up2_taps(gy, HS, y0, y1, wy0, wy1);
    const int c0 = q > 0 ? 2 * q - 1 : 0, c3 = 2 * q + 2 < WS ? 2 * q + 2 : WS - 1;
    const float* r0 = plane + y0 * WS;
    const float* r1 = plane + y1 * WS;
    m0 = *reinterpret_cast<const float2*>(r0 + 2 * q);
    m1 = *reinterpret_cast<const float2*>(r1 + 2 * q);
    a0 = r0[c0];
    a3 = r0[c3];
    b0 = r1[c0];
    b3 = r1[c3];
  }
  __device__ __forceinline__ f32x4 finish(int gy, int q) const {
    int y0, y1;
    float wy0, wy1;
    up2_taps(gy, HS, y0, y1, wy0, wy1);
    const float w0 = q > 0 ? 0.25f : 0.f, w1 = q > 0 ? 0.75f : 1.f;
    f32x4 v;
    v[0] = wy0 * (w0 * a0 + w1 * m0.x) + wy1 * (w0 * b0 + w1 * m1.x);
    v[1] = wy0 * (0.75f * m0.x + 0.25f * m0.y) + wy1 * (0.75f * m1.x + 0.25f * m1.y);
    v[2] = wy0 * (0.25f * m0.x + 0.75f * m0.y) + wy1 * (0.25f * m1.x + 0.75f * m1.y);
    v[3] = wy0 * (0.75f * m0.y + 0.25f * a3) + wy1 * (0.75f * m1.y + 0.25f * b3);
    return v;
  }
};

// A value the compiler cannot prove loop-invariant: keeps the staging index
// math of persistent kernels from being hoisted out of the tile loop (where
// it would hold ~5 VGPRs per staged segment across all the MFMAs).  Used only
// by the full-resolution upsampling convs, whose occupancy it restores; the
// other shapes measured faster with the hoisted (recompute-free) form.
__device__ __forceinline__ int opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// resident blocks per CU x CUs for a persistent launch of kernel k
static int persistent_grid(const void* k, int lds_bytes) {
  int dev = 0, cus = 256, per = 1;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, 256, lds_bytes) != hipSuccess || per < 1) per = 1;
  return per * cus;
}

}  // namespace
