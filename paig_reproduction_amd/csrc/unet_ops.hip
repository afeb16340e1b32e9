// Memory-bound U-Net glue + encoder head kernels (fp32, NCHW per frame):
//   maxpool 2x2 fwd/bwd            nn/network/blocks.py:250,254 (aten max_pool2d)
//   bilinear 2x upsample fwd/bwd   nn/network/blocks.py:260,269 (torchvision Resize,
//                                  == bilinear align_corners=False; antialias no-op)
//   mask softmax + masked objects  nn/network/blocks.py:84-93
//   tanh position head             nn/network/blocks.py:101-102
//   deterministic slab / column reductions for weight and bias gradients.
#include "common.h"

#define PAIG_MAX_SLAB_TASKS 32

namespace {

// ---------------------------------------------------------------- maxpool ----
// The scalar (any-width) kernels are templated on the flat index type: 32-bit
// wherever the element count allows (3bp's 18 / 9-wide levels; 64-bit integer
// division is a long instruction sequence per element)
template <typename I>
__global__ void maxpool_fwd_k(FView x, FViewW y, int F, int C, int H, int W) {
  const int Ho = H / 2, Wo = W / 2;
  const I n = (I)F * C * Ho * Wo;
  for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < n; i += (I)gridDim.x * blockDim.x) {
    int j = i % Wo;
    I t = i / Wo;
    int ii = t % Ho;
    t /= Ho;
    int c = t % C;
    int f = (int)(t / C);
    const float* xp = x.frame(f) + ((long long)c * H + 2 * ii) * W + 2 * j;
    // aten scan order (kh, kw) with "val > max || isnan(val)"
    float m = xp[0];
    float v = xp[1];
    if (v > m || v != v) m = v;
    v = xp[W];
    if (v > m || v != v) m = v;
    v = xp[W + 1];
    if (v > m || v != v) m = v;
    y.frame(f)[((long long)c * Ho + ii) * Wo + j] = m;
  }
}

// dx = (dx_existing + [argmax] * dy) * (x > 0), one thread per input pixel.
template <typename I>
__global__ void maxpool_bwd_relu_k(FView x, FView dy, FViewW dx, int F, int C, int H, int W) {
  const int Ho = H / 2, Wo = W / 2;
  const I n = (I)F * C * H * W;
  for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < n; i += (I)gridDim.x * blockDim.x) {
    int xx = i % W;
    I t = i / W;
    int yy = t % H;
    t /= H;
    int c = t % C;
    int f = (int)(t / C);
    const float* xc = x.frame(f) + (long long)c * H * W;
    float* dxp = dx.frame(f) + (long long)c * H * W + (long long)yy * W + xx;
    float g = *dxp;
    const int pi = yy >> 1, pj = xx >> 1;
    if (pi < Ho && pj < Wo) {
      const float* xp = xc + (2 * pi) * W + 2 * pj;
      int am = 0;
      float m = xp[0];
      float v = xp[1];
      if (v > m || v != v) { m = v; am = 1; }
      v = xp[W];
      if (v > m || v != v) { m = v; am = 2; }
      v = xp[W + 1];
      if (v > m || v != v) { m = v; am = 3; }
      const int me = ((yy & 1) << 1) | (xx & 1);
      if (am == me) g += dy.frame(f)[((long long)c * Ho + pi) * Wo + pj];
    }
    *dxp = xc[(long long)yy * W + xx] > 0.f ? g : 0.f;
  }
}

// Vector forms (W % 4 == 0, H even): one thread per 2 x 2-pooled outputs
// (a 2-row x 4-column input block): float4 loads and stores, 32-bit
// indexing, the argmax computed once per window in aten's scan order.
__device__ __forceinline__ int argmax4(float a, float b, float c, float d, float& m) {
  int am = 0;
  m = a;
  if (b > m || b != b) { m = b; am = 1; }
  if (c > m || c != c) { m = c; am = 2; }
  if (d > m || d != d) { m = d; am = 3; }
  return am;
}

__global__ void maxpool_fwd_v_k(FView x, FViewW y, int F, int C, int H, int W) {
  const int Ho = H / 2, Q = W / 4;
  const int n = F * C * Ho * Q;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int q = i % Q, t = i / Q, pi = t % Ho, fc = t / Ho, c = fc % C, f = fc / C;
    const float* xp = x.frame(f) + ((long long)c * H + 2 * pi) * W + 4 * q;
    const float4 a = *reinterpret_cast<const float4*>(xp);
    const float4 b = *reinterpret_cast<const float4*>(xp + W);
    float m0, m1;
    argmax4(a.x, a.y, b.x, b.y, m0);
    argmax4(a.z, a.w, b.z, b.w, m1);
    *reinterpret_cast<float2*>(y.frame(f) + ((long long)c * Ho + pi) * (W / 2) + 2 * q) = make_float2(m0, m1);
  }
}

// The standalone pool's forward for a layer whose backward folds the pool
// (paig_conv2d_bwd flags & 64) where the conv's forward cannot pool in its
// epilogue (rows not whole 16-pixel M-tiles: 3bp's 36 / 18): the pooled
// values (maxpool_fwd_k's scan order, bit-identical) and one code byte per
// (channel, window) in the layout the fused pool writes (conv_split.hip
// pool_code): ReLU' bits of the window's pixels (y, x), (y, x+1), (y+1, x),
// (y+1, x+1) in bits 0..3, the argmax in bits 4..5; [C/8][H/2][W/2][C%8]
__global__ void maxpool_fwd_codes_k(FView x, FViewW y, unsigned char* __restrict__ code, long long code_fs, int F, int C,
                                    int H, int W) {
  const int Ho = H / 2, Wo = W / 2;
  const int n = F * C * Ho * Wo;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int j = i % Wo, t = i / Wo, pi = t % Ho, fc = t / Ho, c = fc % C, f = fc / C;
    const float* xp = x.frame(f) + ((long long)c * H + 2 * pi) * W + 2 * j;
    const float a = xp[0], b = xp[1], cc = xp[W], d = xp[W + 1];
    float m;
    const int am = argmax4(a, b, cc, d, m);
    y.frame(f)[((long long)c * Ho + pi) * Wo + j] = m;
    code[(long long)f * code_fs + (((long long)(c >> 3) * Ho + pi) * Wo + j) * 8 + (c & 7)] =
        (unsigned char)((a > 0.f ? 1 : 0) | (b > 0.f ? 2 : 0) | (cc > 0.f ? 4 : 0) | (d > 0.f ? 8 : 0) | (am << 4));
  }
}

// dx = (dx + [argmax] * dy) * (x > 0)
__global__ void maxpool_bwd_relu_v_k(FView x, FView dy, FViewW dx, int F, int C, int H, int W) {
  const int Ho = H / 2, Q = W / 4;
  const int n = F * C * Ho * Q;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int q = i % Q, t = i / Q, pi = t % Ho, fc = t / Ho, c = fc % C, f = fc / C;
    const long long o = ((long long)c * H + 2 * pi) * W + 4 * q;
    const float* xp = x.frame(f) + o;
    float* dp = dx.frame(f) + o;
    const float4 a = *reinterpret_cast<const float4*>(xp);
    const float4 b = *reinterpret_cast<const float4*>(xp + W);
    const float2 g = *reinterpret_cast<const float2*>(dy.frame(f) + ((long long)c * Ho + pi) * (W / 2) + 2 * q);
    float4 d0 = *reinterpret_cast<const float4*>(dp);
    float4 d1 = *reinterpret_cast<const float4*>(dp + W);
    float m;
    const int a0 = argmax4(a.x, a.y, b.x, b.y, m);
    const int a1 = argmax4(a.z, a.w, b.z, b.w, m);
    if (a0 == 0) d0.x += g.x; else if (a0 == 1) d0.y += g.x; else if (a0 == 2) d1.x += g.x; else d1.y += g.x;
    if (a1 == 0) d0.z += g.y; else if (a1 == 1) d0.w += g.y; else if (a1 == 2) d1.z += g.y; else d1.w += g.y;
    d0.x = a.x > 0.f ? d0.x : 0.f;
    d0.y = a.y > 0.f ? d0.y : 0.f;
    d0.z = a.z > 0.f ? d0.z : 0.f;
    d0.w = a.w > 0.f ? d0.w : 0.f;
    d1.x = b.x > 0.f ? d1.x : 0.f;
    d1.y = b.y > 0.f ? d1.y : 0.f;
    d1.z = b.z > 0.f ? d1.z : 0.f;
    d1.w = b.w > 0.f ? d1.w : 0.f;
    *reinterpret_cast<float4*>(dp) = d0;
    *reinterpret_cast<float4*>(dp + W) = d1;
  }
}

// ------------------------------------------------------- bilinear upsample ---
// 1-D taps of aten's upsample_bilinear2d (align_corners=False, no scale given):
//   src = max(0, (dst + 0.5) * in/out - 0.5); i0 = floor(src); i1 = min(i0+1, in-1)
__device__ __forceinline__ void up_taps(int dst, int in, int out, int& i0, int& i1, float& l0, float& l1) {
  const float scale = (float)in / (float)out;
  float s = scale * ((float)dst + 0.5f) - 0.5f;
  if (s < 0.f) s = 0.f;
  i0 = (int)s;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = s - (float)i0;
  l0 = 1.f - l1;
}

template <typename I>
__global__ void upsample_fwd_k(FView s, FViewW u, int F, int C, int Hs, int Ws, int Ho, int Wo) {
  const I n = (I)F * C * Ho * Wo;
  for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < n; i += (I)gridDim.x * blockDim.x) {
    int x = i % Wo;
    I t = i / Wo;
    int y = t % Ho;
    t /= Ho;
    int c = t % C;
    int f = (int)(t / C);
    int y0, y1, x0, x1;
    float wy0, wy1, wx0, wx1;
    up_taps(y, Hs, Ho, y0, y1, wy0, wy1);
    up_taps(x, Ws, Wo, x0, x1, wx0, wx1);
    const float* sp = s.frame(f) + (long long)c * Hs * Ws;
    float v = wy0 * (wx0 * sp[y0 * Ws + x0] + wx1 * sp[y0 * Ws + x1]) +
              wy1 * (wx0 * sp[y1 * Ws + x0] + wx1 * sp[y1 * Ws + x1]);
    u.frame(f)[((long long)c * Ho + y) * Wo + x] = v;
  }
}

// ds[sy][sx] = sum over outputs using it (gather form, deterministic), then
// optionally * (s > 0) (ReLU'd source).
template <typename I>
__global__ void upsample_bwd_k(FView du, FView s, FViewW ds, int F, int C, int Hs, int Ws, int Ho, int Wo,
                               int relu_mask) {
  const I n = (I)F * C * Hs * Ws;
  for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < n; i += (I)gridDim.x * blockDim.x) {
    int sx = i % Ws;
    I t = i / Ws;
    int sy = t % Hs;
    t /= Hs;
    int c = t % C;
    int f = (int)(t / C);
    const float* dup = du.frame(f) + (long long)c * Ho * Wo;
    // exact 2x: source s receives from outputs 2s-1 .. 2s+2 with weights
    // 1/4, 3/4, 3/4, 1/4 (the clamped edges give 1 to s = 0 from 0 and to
    // s = n-1 from 2n-1) -- the same, exactly representable taps as up_taps
    float wy[4], wx[4];
    wy[0] = sy >= 1 ? 0.25f : 0.f;
    wy[1] = sy == 0 ? 1.f : 0.75f;
    wy[2] = sy == Hs - 1 ? 1.f : 0.75f;
    wy[3] = sy <= Hs - 2 ? 0.25f : 0.f;
    wx[0] = sx >= 1 ? 0.25f : 0.f;
    wx[1] = sx == 0 ? 1.f : 0.75f;
    wx[2] = sx == Ws - 1 ? 1.f : 0.75f;
    wx[3] = sx <= Ws - 2 ? 0.25f : 0.f;
    float acc = 0.f;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int y = 2 * sy - 1 + a;
      if (wy[a] == 0.f) continue;
      const float* rp = dup + y * Wo;
      float row = 0.f;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int x = 2 * sx - 1 + b;
        if (wx[b] != 0.f) row = fmaf(wx[b], rp[x], row);
      }
      acc = fmaf(wy[a], row, acc);
    }
    if (relu_mask) acc = s.frame(f)[((long long)c * Hs + sy) * Ws + sx] > 0.f ? acc : 0.f;
    ds.frame(f)[((long long)c * Hs + sy) * Ws + sx] = acc;
  }
}

// Vector form (Ws even): one thread per 2 horizontally adjacent source
// pixels; each reads its 4 du rows as float4 + 2 edge scalars.  The per-pixel
// accumulation order (and the zero-weight taps, which add exact zeros) is the
// scalar kernel's, so the two forms agree bit for bit on finite inputs.
__global__ void upsample_bwd_v_k(FView du, FView s, FViewW ds, int F, int C, int Hs, int Ws, int relu_mask) {
  const int Ho = 2 * Hs, Wo = 2 * Ws, P = Ws / 2;
  const int n = F * C * Hs * P;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int m = i % P, t = i / P, sy = t % Hs, fc = t / Hs, c = fc % C, f = fc / C;
    const float* dup = du.frame(f) + (long long)c * Ho * Wo;
    float wy[4];
    wy[0] = sy >= 1 ? 0.25f : 0.f;
    wy[1] = sy == 0 ? 1.f : 0.75f;
    wy[2] = sy == Hs - 1 ? 1.f : 0.75f;
    wy[3] = sy <= Hs - 2 ? 0.25f : 0.f;
    // source columns sx0 = 2m, sx1 = 2m + 1 read du columns 4m-1 .. 4m+4
    const int s0 = 2 * m, s1 = 2 * m + 1;
    float wx0[4], wx1[4];
    wx0[0] = s0 >= 1 ? 0.25f : 0.f;
    wx0[1] = s0 == 0 ? 1.f : 0.75f;
    wx0[2] = s0 == Ws - 1 ? 1.f : 0.75f;
    wx0[3] = s0 <= Ws - 2 ? 0.25f : 0.f;
    wx1[0] = 0.25f;
    wx1[1] = 0.75f;
    wx1[2] = s1 == Ws - 1 ? 1.f : 0.75f;
    wx1[3] = s1 <= Ws - 2 ? 0.25f : 0.f;
    float acc0 = 0.f, acc1 = 0.f;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int y = 2 * sy - 1 + a;
      if (wy[a] == 0.f) continue;
      const float* rp = dup + y * Wo + 4 * m;
      const float4 v = *reinterpret_cast<const float4*>(rp);
      // the edge columns 4m-1 / 4m+4 are the neighbouring lanes' float4 ends
      // when a row's P lanes never straddle a wave (P divides 64): lanes i-1 /
      // i+1 hold m-1 / m+1 of the same row wherever those taps carry weight
      // (at m = 0 and m = P-1 the weight is zero); else two scalar loads
      float l, r;
      if (64 % P == 0) {
        l = __shfl_up(v.w, 1, 64);
        r = __shfl_down(v.x, 1, 64);
      } else {
        l = m > 0 ? rp[-1] : 0.f;
        r = 4 * m + 4 < Wo ? rp[4] : 0.f;
      }
      float row0 = 0.f, row1 = 0.f;
      if (wx0[0] != 0.f) row0 = fmaf(wx0[0], l, row0);
      row0 = fmaf(wx0[1], v.x, row0);
      row0 = fmaf(wx0[2], v.y, row0);
      if (wx0[3] != 0.f) row0 = fmaf(wx0[3], v.z, row0);
      row1 = fmaf(wx1[0], v.y, row1);
      row1 = fmaf(wx1[1], v.z, row1);
      row1 = fmaf(wx1[2], v.w, row1);
      if (wx1[3] != 0.f) row1 = fmaf(wx1[3], r, row1);
      acc0 = fmaf(wy[a], row0, acc0);
      acc1 = fmaf(wy[a], row1, acc1);
    }
    const long long so = ((long long)c * Hs + sy) * Ws + 2 * m;
    if (relu_mask) {
      const float2 sv = *reinterpret_cast<const float2*>(s.frame(f) + so);
      acc0 = sv.x > 0.f ? acc0 : 0.f;
      acc1 = sv.y > 0.f ? acc1 : 0.f;
    }
    *reinterpret_cast<float2*>(ds.frame(f) + so) = make_float2(acc0, acc1);
  }
}

// ------------------------------------------------------------ mask softmax ---
// logits [F][K][HW] (ReLU'd U-Net output) ++ constant 1 (background) ->
// masks [F][K+1][HW]; masked objects A[k*F + f][c*HW + p] = mask_k * x[f][c][p].
__global__ void mask_softmax_fwd_k(const float* __restrict__ lg, FView x, float* __restrict__ masks,
                                   float* __restrict__ objs, int F, int K, int C, int HW) {
  const long long n = (long long)F * HW;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int p = i % HW;
    const int f = (int)(i / HW);
    float l[8];
    float m = 1.f;
    for (int k = 0; k < K; ++k) {
      l[k] = lg[((long long)f * K + k) * HW + p];
      m = fmaxf(m, l[k]);
    }
    float e[9];
    float s = 0.f;
    for (int k = 0; k < K; ++k) {
      e[k] = expf(l[k] - m);
      s += e[k];
    }
    e[K] = expf(1.f - m);
    s += e[K];
    const float* xp = x.frame(f);
    for (int k = 0; k <= K; ++k) {
      const float mk = e[k] / s;
      masks[((long long)f * (K + 1) + k) * HW + p] = mk;
      if (k < K)
        for (int c = 0; c < C; ++c) objs[((long long)k * F + f) * C * HW + (long long)c * HW + p] = mk * xp[c * HW + p];
    }
  }
}

// UNet (H >= 40): the same softmax over 2x2 quads, also writing the
// AvgPool2d(2) of the masked objects that feeds l1 (blocks.py:94-96); window
// sum in aten's (0,0),(0,1),(1,0),(1,1) order, then * 1/4 (exact).
__global__ void mask_softmax_pool_fwd_k(const float* __restrict__ lg, FView x, float* __restrict__ masks,
                                        float* __restrict__ objs, float* __restrict__ pobjs, int F, int K, int C,
                                        int H, int W) {
  const int H2 = H / 2, W2 = W / 2, HW = H * W, HW4 = H2 * W2;
  const long long n = (long long)F * HW4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int q = (int)(i % HW4);
    const int f = (int)(i / HW4);
    const int qy = q / W2, qx = q % W2;
    const float* xp = x.frame(f);
    float acc[7][3];
    for (int k = 0; k < K; ++k)
      for (int c = 0; c < 3; ++c) acc[k][c] = 0.f;
    for (int d = 0; d < 4; ++d) {
      const int p = (2 * qy + (d >> 1)) * W + 2 * qx + (d & 1);
      float l[8];
      float m = 1.f;
      for (int k = 0; k < K; ++k) {
        l[k] = lg[((long long)f * K + k) * HW + p];
        m = fmaxf(m, l[k]);
      }
      float e[9];
      float s = 0.f;
      for (int k = 0; k < K; ++k) {
        e[k] = expf(l[k] - m);
        s += e[k];
      }
      e[K] = expf(1.f - m);
      s += e[K];
      for (int k = 0; k <= K; ++k) {
        const float mk = e[k] / s;
        masks[((long long)f * (K + 1) + k) * HW + p] = mk;
        if (k < K)
          for (int c = 0; c < C; ++c) {
            const float o = mk * xp[c * HW + p];
            objs[((long long)k * F + f) * C * HW + (long long)c * HW + p] = o;
            acc[k][c] += o;
          }
      }
    }
    for (int k = 0; k < K; ++k)
      for (int c = 0; c < C; ++c) pobjs[((long long)k * F + f) * C * HW4 + (long long)c * HW4 + q] = acc[k][c] * 0.25f;
  }
}

// dlogits[f][k][p] = [relu'(lg)] * m_k * (dm_k - sum_j m_j dm_j),
// dm_k = sum_c dobjs[k*F+f][c][p] * x[f][c][p] (k < K), dm_bg = 0.
// flags: 1 the logits are ReLU'd (ShallowUNet c13, Q13), 2 dobjs is the
// gradient of the 2x2-average-pooled objects (UNet: d = dpooled / 4).
__global__ void mask_softmax_bwd_k(const float* __restrict__ lg, FView x, const float* __restrict__ masks,
                                   const float* __restrict__ dobjs, float* __restrict__ dlg, int F, int K, int C,
                                   int H, int W, int flags) {
  const int HW = H * W;
  const bool pooled = (flags & 2) != 0;
  const int W2 = W / 2, HW4 = (H / 2) * W2;
  const long long n = (long long)F * HW;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int p = i % HW;
    const int f = (int)(i / HW);
    const float* xp = x.frame(f);
    const int pq = pooled ? ((p / W) >> 1) * W2 + ((p % W) >> 1) : p;
    const int DHW = pooled ? HW4 : HW;
    float dm[8], mk[8];
    float dot = 0.f;
    for (int k = 0; k < K; ++k) {
      float a = 0.f;
      for (int c = 0; c < C; ++c) {
        float d = dobjs[((long long)k * F + f) * C * DHW + (long long)c * DHW + pq];
        if (pooled) d *= 0.25f;
        a = fmaf(d, xp[c * HW + p], a);
      }
      dm[k] = a;
      mk[k] = masks[((long long)f * (K + 1) + k) * HW + p];
      dot = fmaf(mk[k], a, dot);
    }
    for (int k = 0; k < K; ++k) {
      const float g = mk[k] * (dm[k] - dot);
      dlg[((long long)f * K + k) * HW + p] = ((flags & 1) && !(lg[((long long)f * K + k) * HW + p] > 0.f)) ? 0.f : g;
    }
  }
}

// The same, 4 pixels per thread (float4 loads and stores; frames of HW % 4
// == 0 pixels, K a template constant): per element the scalar kernel's
// operation order, so the results are identical.
typedef float m4 __attribute__((ext_vector_type(4)));
template <int K>
__global__ void mask_softmax_fwd_v_k(const float* __restrict__ lg, FView x, float* __restrict__ masks,
                                     float* __restrict__ objs, int F, int C, int HW) {
  const int Q = HW / 4;
  const long long n = (long long)F * Q;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int p = (int)(i % Q) * 4;
    const int f = (int)(i / Q);
    m4 l[K], e[K + 1];
    m4 m = m4{1.f, 1.f, 1.f, 1.f};
#pragma unroll
    for (int k = 0; k < K; ++k) {
      l[k] = *reinterpret_cast<const m4*>(lg + ((long long)f * K + k) * HW + p);
#pragma unroll
      for (int j = 0; j < 4; ++j) m[j] = fmaxf(m[j], l[k][j]);
    }
    m4 s = m4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < K; ++k) {
#pragma unroll
      for (int j = 0; j < 4; ++j) e[k][j] = expf(l[k][j] - m[j]);
      s += e[k];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) e[K][j] = expf(1.f - m[j]);
    s += e[K];
    const float* xp = x.frame(f);
    m4 xv[3];
#pragma unroll
    for (int c = 0; c < 3; ++c)
      if (c < C) xv[c] = *reinterpret_cast<const m4*>(xp + c * HW + p);
#pragma unroll
    for (int k = 0; k <= K; ++k) {
      m4 mk;
#pragma unroll
      for (int j = 0; j < 4; ++j) mk[j] = e[k][j] / s[j];
      *reinterpret_cast<m4*>(masks + ((long long)f * (K + 1) + k) * HW + p) = mk;
      if (k < K)
#pragma unroll
        for (int c = 0; c < 3; ++c)
          if (c < C) *reinterpret_cast<m4*>(objs + ((long long)k * F + f) * C * HW + (long long)c * HW + p) = mk * xv[c];
    }
  }
}

template <int K>
__global__ void mask_softmax_bwd_v_k(const float* __restrict__ lg, FView x, const float* __restrict__ masks,
                                     const float* __restrict__ dobjs, float* __restrict__ dlg, int F, int C, int HW,
                                     int flags) {
  const int Q = HW / 4;
  const long long n = (long long)F * Q;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int p = (int)(i % Q) * 4;
    const int f = (int)(i / Q);
    const float* xp = x.frame(f);
    m4 xv[3];
#pragma unroll
    for (int c = 0; c < 3; ++c)
      if (c < C) xv[c] = *reinterpret_cast<const m4*>(xp + c * HW + p);
    m4 dm[K], mk[K];
    m4 dot = m4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < K; ++k) {
      m4 a = m4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 3; ++c)
        if (c < C) {
          const m4 d = *reinterpret_cast<const m4*>(dobjs + ((long long)k * F + f) * C * HW + (long long)c * HW + p);
#pragma unroll
          for (int j = 0; j < 4; ++j) a[j] = fmaf(d[j], xv[c][j], a[j]);
        }
      dm[k] = a;
      mk[k] = *reinterpret_cast<const m4*>(masks + ((long long)f * (K + 1) + k) * HW + p);
#pragma unroll
      for (int j = 0; j < 4; ++j) dot[j] = fmaf(mk[k][j], a[j], dot[j]);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      m4 g = mk[k] * (dm[k] - dot);
      if (flags & 1) {
        const m4 lv = *reinterpret_cast<const m4*>(lg + ((long long)f * K + k) * HW + p);
#pragma unroll
        for (int j = 0; j < 4; ++j) g[j] = lv[j] > 0.f ? g[j] : 0.f;
      }
      *reinterpret_cast<m4*>(dlg + ((long long)f * K + k) * HW + p) = g;
    }
  }
}

// ------------------------------------------- fused U-Net head + mask softmax ----
// The U-Net's last layer (a 1x1 conv, CI -> K) fused into the mask softmax
// (blocks.py:84-96): the logits are formed per pixel in fp32 FMAs from the
// previous layer's output and never stored.
//   * ShallowUNet (H < 40): c13, 8 -> K, ReLU'd (Q13; blocks.py:276,307);
//   * UNet (H >= 40): c18, 16 -> K, not ReLU'd (blocks.py:170,236), and the
//     masked objects' AvgPool2d(2) (blocks.py:94-96) that feeds l1.
// Forward: logits -> softmax -> masks, masked objects (+ pooled objects).
// Backward: the softmax backward (from the pooled objects' gradient on the
// UNet), the ReLU' of the logits where they are ReLU'd (recomputed in the
// forward's exact operation order), the head's input gradient with the
// previous layer's ReLU' (dXl: that layer's dY) and the head's weight / bias
// gradient as one slab row per block (deterministic order, reduced with the
// U-Net's slabs).  Replaces the head conv's forward / dgrad / wgrad and the
// separate softmax kernels: the logits' write and re-reads and 3 launches
// (mnist: 1.05 ms per step of separate kernels).
template <int K, int CI>
__device__ __forceinline__ void head_logits(const float* __restrict__ w, const float* __restrict__ b, const m4* xv,
                                            m4* l) {
#pragma unroll
  for (int k = 0; k < K; ++k) {
    m4 a = m4{b[k], b[k], b[k], b[k]};
#pragma unroll
    for (int c = 0; c < CI; ++c)
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = fmaf(w[k * CI + c], xv[c][j], a[j]);
    l[k] = a;
  }
}

// logits -> (ReLU) -> softmax with the constant background logit 1, in
// mask_softmax_fwd_v_k's operation order: mk[0..K] (4 pixels each)
template <int K, bool RELU>
__device__ __forceinline__ void head_softmax(m4* l, m4* mk) {
  m4 m = m4{1.f, 1.f, 1.f, 1.f}, e[K + 1];
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (RELU) l[k][j] = l[k][j] < 0.f ? 0.f : l[k][j];   // c13's ReLU (Q13)
      m[j] = fmaxf(m[j], l[k][j]);
    }
  m4 s = m4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < K; ++k) {
#pragma unroll
    for (int j = 0; j < 4; ++j) e[k][j] = expf(l[k][j] - m[j]);
    s += e[k];
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) e[K][j] = expf(1.f - m[j]);
  s += e[K];
#pragma unroll
  for (int k = 0; k <= K; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) mk[k][j] = e[k][j] / s[j];
}

template <int K, int CI, bool RELU>
__global__ void __launch_bounds__(256) head_mask_fwd_k(const float* __restrict__ xl, const float* __restrict__ w,
                                                       const float* __restrict__ b, FView x, float* __restrict__ masks,
                                                       float* __restrict__ objs, int F, int HW) {
  const int Q = HW / 4;
  const long long n = (long long)F * Q;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int p = (int)(i % Q) * 4;
    const int f = (int)(i / Q);
    m4 hv[CI];
#pragma unroll
    for (int c = 0; c < CI; ++c) hv[c] = *reinterpret_cast<const m4*>(xl + ((long long)f * CI + c) * HW + p);
    const float* xp = x.frame(f);
    m4 xv[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) xv[c] = *reinterpret_cast<const m4*>(xp + c * HW + p);
    m4 l[K], mk[K + 1];
    head_logits<K, CI>(w, b, hv, l);
    head_softmax<K, RELU>(l, mk);
#pragma unroll
    for (int k = 0; k <= K; ++k) {
      *reinterpret_cast<m4*>(masks + ((long long)f * (K + 1) + k) * HW + p) = mk[k];
      if (k < K)
#pragma unroll
        for (int c = 0; c < 3; ++c)
          *reinterpret_cast<m4*>(objs + ((long long)k * F + f) * 3 * HW + (long long)c * HW + p) = mk[k] * xv[c];
    }
  }
}

// UNet: item = columns 4u .. 4u+3 of the row pair 2py, 2py+1 (two 2x2
// windows): masks and objects of both rows, and the windows' average in
// mask_softmax_pool_fwd_k's order ((0,0), (0,1), (1,0), (1,1), then * 1/4)
template <int K, int CI, bool RELU>
__global__ void __launch_bounds__(256) head_mask_pool_fwd_k(const float* __restrict__ xl, const float* __restrict__ w,
                                                            const float* __restrict__ b, FView x,
                                                            float* __restrict__ masks, float* __restrict__ objs,
                                                            float* __restrict__ pobjs, int F, int H, int W) {
  const int HW = H * W, W2 = W / 2, W4 = W / 4, HW4 = (H / 2) * W2;
  const long long n = (long long)F * (H / 2) * W4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int u = (int)(i % W4), py = (int)((i / W4) % (H / 2)), f = (int)(i / ((long long)W4 * (H / 2)));
    const float* xp = x.frame(f);
    float2 pa[K][3];
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int c = 0; c < 3; ++c) pa[k][c] = make_float2(0.f, 0.f);
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      const int p = (2 * py + rr) * W + 4 * u;
      m4 hv[CI];
#pragma unroll
      for (int c = 0; c < CI; ++c) hv[c] = *reinterpret_cast<const m4*>(xl + ((long long)f * CI + c) * HW + p);
      m4 xv[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) xv[c] = *reinterpret_cast<const m4*>(xp + c * HW + p);
      m4 l[K], mk[K + 1];
      head_logits<K, CI>(w, b, hv, l);
      head_softmax<K, RELU>(l, mk);
#pragma unroll
      for (int k = 0; k <= K; ++k) {
        *reinterpret_cast<m4*>(masks + ((long long)f * (K + 1) + k) * HW + p) = mk[k];
        if (k < K)
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const m4 o = mk[k] * xv[c];
            *reinterpret_cast<m4*>(objs + ((long long)k * F + f) * 3 * HW + (long long)c * HW + p) = o;
            pa[k][c].x += o[0];
            pa[k][c].x += o[1];
            pa[k][c].y += o[2];
            pa[k][c].y += o[3];
          }
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int c = 0; c < 3; ++c)
        *reinterpret_cast<float2*>(pobjs + ((long long)k * F + f) * 3 * HW4 + (long long)c * HW4 + py * W2 + 2 * u) =
            make_float2(pa[k][c].x * 0.25f, pa[k][c].y * 0.25f);
  }
}

// POOL: dobjs is the gradient of the pooled objects [K][F][3][H/2][W/2]
// (each pixel takes 1/4 of its window's, mask_softmax_bwd_k's order)
template <int K, int CI, bool RELU, bool POOL>
__global__ void __launch_bounds__(256) head_mask_bwd_k(const float* __restrict__ xl, const float* __restrict__ w,
                                                       const float* __restrict__ b, FView x,
                                                       const float* __restrict__ masks, const float* __restrict__ dobjs,
                                                       float* __restrict__ dxl, float* __restrict__ slab, int F, int H,
                                                       int W) {
  constexpr int NW = K * CI + K;   // slab row: dW[k][c], then db[k]
  const int HW = H * W, W2 = W / 2, HW4 = (H / 2) * W2;
  const int DHW = POOL ? HW4 : HW;
  const int Q = HW / 4;
  const long long n = (long long)F * Q;
  float acc[NW];
#pragma unroll
  for (int t = 0; t < NW; ++t) acc[t] = 0.f;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int p = (int)(i % Q) * 4;
    const int f = (int)(i / Q);
    const int pq = POOL ? ((p / W) >> 1) * W2 + ((p % W) >> 1) : p;   // (pooled) index of the first pixel
    m4 hv[CI];
#pragma unroll
    for (int c = 0; c < CI; ++c) hv[c] = *reinterpret_cast<const m4*>(xl + ((long long)f * CI + c) * HW + p);
    const float* xp = x.frame(f);
    m4 xv[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) xv[c] = *reinterpret_cast<const m4*>(xp + c * HW + p);
    // softmax backward (mask_softmax_bwd_v_k's / mask_softmax_bwd_k's order)
    m4 dm[K], mk[K];
    m4 dot = m4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < K; ++k) {
      m4 a = m4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float* dp = dobjs + ((long long)k * F + f) * 3 * DHW + (long long)c * DHW + pq;
        m4 d;
        if constexpr (POOL) {
          const float2 dq = *reinterpret_cast<const float2*>(dp);
          d = m4{dq.x, dq.x, dq.y, dq.y} * 0.25f;
        } else {
          d = *reinterpret_cast<const m4*>(dp);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] = fmaf(d[j], xv[c][j], a[j]);
      }
      dm[k] = a;
      mk[k] = *reinterpret_cast<const m4*>(masks + ((long long)f * (K + 1) + k) * HW + p);
#pragma unroll
      for (int j = 0; j < 4; ++j) dot[j] = fmaf(mk[k][j], a[j], dot[j]);
    }
    m4 g[K];
    if constexpr (RELU) {
      m4 l[K];
      head_logits<K, CI>(w, b, hv, l);
#pragma unroll
      for (int k = 0; k < K; ++k) {
        g[k] = mk[k] * (dm[k] - dot);
#pragma unroll
        for (int j = 0; j < 4; ++j) g[k][j] = l[k][j] > 0.f ? g[k][j] : 0.f;   // c13's ReLU'
      }
    } else {
#pragma unroll
      for (int k = 0; k < K; ++k) g[k] = mk[k] * (dm[k] - dot);
    }
    // the head's input gradient (the previous layer's ReLU' applied) and the
    // weight / bias partials
#pragma unroll
    for (int c = 0; c < CI; ++c) {
      m4 d = m4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int j = 0; j < 4; ++j) d[j] = fmaf(w[k * CI + c], g[k][j], d[j]);
#pragma unroll
      for (int j = 0; j < 4; ++j) d[j] = hv[c][j] > 0.f ? d[j] : 0.f;
      *reinterpret_cast<m4*>(dxl + ((long long)f * CI + c) * HW + p) = d;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
#pragma unroll
      for (int c = 0; c < CI; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[k * CI + c] = fmaf(g[k][j], hv[c][j], acc[k * CI + c]);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[K * CI + k] += g[k][j];
    }
  }
  // block reduction in a fixed order: wave butterflies, then the 4 waves
  __shared__ float red[4][NW];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int t = 0; t < NW; ++t) {
    float v = acc[t];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[wv][t] = v;
  }
  __syncthreads();
  if (threadIdx.x < NW)
    slab[(long long)blockIdx.x * NW + threadIdx.x] =
        ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
}

// --------------------------------------------------------- position head ----
// enc_pos[n][2k+j] = tanh(h3[k*N+n][j]) * (H/2) + H/2
__global__ void pos_head_fwd_k(const float* __restrict__ h3, float* __restrict__ pos, int N, int K, float half) {
  const int n = N * K * 2;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int j = i & 1;
    const int k = (i >> 1) % K;
    const int r = i / (2 * K);
    pos[i] = tanhf(h3[((long long)k * N + r) * 2 + j]) * half + half;
  }
}

__global__ void pos_head_bwd_k(const float* __restrict__ h3, const float* __restrict__ dpos, float* __restrict__ dh3,
                               int N, int K, float half) {
  const int n = N * K * 2;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int j = i & 1;
    const int k = (i >> 1) % K;
    const int r = i / (2 * K);
    const long long o = ((long long)k * N + r) * 2 + j;
    const float t = tanhf(h3[o]);
    dh3[o] = dpos[i] * half * (1.f - t * t);
  }
}

// ------------------------------------------------------- velocity packing ----
// enc_pos [B][Te][D] (D = 2K). Forward (blocks.py:43-45, non-alt):
//   X[k*B+b][t*2+j] = pos[b][t][2k+j], t < S
// alt_vel (blocks.py:33-38): X[k*B+b][t*2+j] = pos[b][t+1][2k+j] - pos[b][t][2k+j], t < S-1
__global__ void vel_pack_k(const float* __restrict__ pos, float* __restrict__ X, int B, int Te, int K, int S,
                           int alt) {
  const int cols = (alt ? S - 1 : S) * 2;
  const int n = K * B * cols;
  const int D = 2 * K;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int col = i % cols;
    const int row = i / cols;
    const int k = row / B, b = row % B;
    const int t = col >> 1, j = col & 1;
    const float* pb = pos + (long long)b * Te * D + 2 * k + j;
    X[i] = alt ? pb[(t + 1) * D] - pb[t * D] : pb[t * D];
  }
}

// dpos[b][t][2k+j] += dX (+ dpos0[b][2k+j] at t = S-1 where dpos0 != null).
// One thread per (b, t, d) of the first S steps: no write conflicts.
__global__ void vel_unpack_add_k(const float* __restrict__ dX, const float* __restrict__ dpos0, float* __restrict__ dpos,
                                 int B, int Te, int K, int S, int alt) {
  const int D = 2 * K;
  const int cols = (alt ? S - 1 : S) * 2;
  const int n = B * S * D;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int d = i % D;
    const int t = (i / D) % S;
    const int b = i / (D * S);
    const int k = d >> 1, j = d & 1;
    const float* xr = dX ? dX + (long long)(k * B + b) * cols : nullptr;
    float g = 0.f;
    if (xr) {
      if (alt) {
        if (t >= 1) g += xr[(t - 1) * 2 + j];
        if (t <= S - 2) g -= xr[t * 2 + j];
      } else {
        g += xr[t * 2 + j];
      }
    }
    if (dpos0 && t == S - 1) g += dpos0[(long long)b * D + d];
    dpos[((long long)b * Te + t) * D + d] += g;
  }
}

// ------------------------------------------------------------- reductions ---
// out[i] (+)= sum_b slab[b][i]; 64 columns per block, 4 waves split the rows.
__global__ void __launch_bounds__(256) slab_reduce_k(const float* __restrict__ slab, int nblk, long long ld, int len,
                                                     float* __restrict__ out, int accumulate) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (i < len)
    for (int b = wv; b < nblk; b += 4) s += slab[(long long)b * ld + i];
  red[wv][lane] = s;
  __syncthreads();
  if (wv == 0 && i < len) {
    float v = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    out[i] = accumulate ? out[i] + v : v;
  }
}

// Many reductions in one launch: task t sums nblk[t] rows of len[t] floats
// (row stride len[t]) into dst[t]; blocks [start[t], start[t+1]) serve task t.
struct SlabTasks {
  const float* src[PAIG_MAX_SLAB_TASKS];
  float* dst[PAIG_MAX_SLAB_TASKS];
  int nblk[PAIG_MAX_SLAB_TASKS];
  int len[PAIG_MAX_SLAB_TASKS];
  int vec[PAIG_MAX_SLAB_TASKS];  // 1: len % 4 == 0 and src/dst 16-B aligned -> float4 path
  int start[PAIG_MAX_SLAB_TASKS + 1];
  int ntask;
  int accumulate;
};

// Scalar path (64 columns per block): 16 waves, each lane owns one column,
// the waves stride the rows (4 independent accumulators each), then a
// fixed-order combine.
__device__ __forceinline__ void slab_cols_scalar(const float* __restrict__ src, float* dst, int len, int nblk,
                                                 int blk, int accumulate, float (*red)[64]) {
  constexpr int NW = 16;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int i = blk * 64 + lane;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (i < len) {
    int b = wv;
    for (; b + 3 * NW < nblk; b += 4 * NW) {
      s0 += src[(long long)b * len + i];
      s1 += src[(long long)(b + NW) * len + i];
      s2 += src[(long long)(b + 2 * NW) * len + i];
      s3 += src[(long long)(b + 3 * NW) * len + i];
    }
    for (; b < nblk; b += NW) s0 += src[(long long)b * len + i];
  }
  red[wv][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (wv == 0 && i < len) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[w][lane];
    dst[i] = accumulate ? dst[i] + v : v;
  }
}

// Vector path (32 columns per block): 8 lanes x float4 cover one 128-B row
// segment, so a wave reads 8 rows per instruction and a task gets twice the
// blocks of the scalar path (the decoder's 5 K-column source reduction:
// 80 -> 160 CUs busy, 11 -> 7.5 us).  Rows r, r+128, ... go to row lane r; a
// fixed-shape LDS tree combines the 128 row lanes, so the order is the same
// every run.
__device__ __forceinline__ void slab_cols_vec(const float* __restrict__ src0, float* dst, int len, int nblk, int blk,
                                              int accumulate, float4 (*red)[8]) {
  constexpr int NR = 128;
  const int c4 = threadIdx.x & 7, r = threadIdx.x >> 3;
  const int col = blk * 32 + c4 * 4;
  float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
  if (col < len) {
    const float* src = src0 + col;
    int b = r;
    for (; b + NR < nblk; b += 2 * NR) {
      const float4 a = *reinterpret_cast<const float4*>(src + (long long)b * len);
      const float4 c = *reinterpret_cast<const float4*>(src + (long long)(b + NR) * len);
      s0.x += a.x; s0.y += a.y; s0.z += a.z; s0.w += a.w;
      s1.x += c.x; s1.y += c.y; s1.z += c.z; s1.w += c.w;
    }
    if (b < nblk) {
      const float4 a = *reinterpret_cast<const float4*>(src + (long long)b * len);
      s0.x += a.x; s0.y += a.y; s0.z += a.z; s0.w += a.w;
    }
  }
  red[r][c4] = make_float4(s0.x + s1.x, s0.y + s1.y, s0.z + s1.z, s0.w + s1.w);
  __syncthreads();
#pragma unroll
  for (int h = NR / 2; h >= 1; h >>= 1) {
    if (r < h) {
      const float4 a = red[r][c4], c = red[r + h][c4];
      red[r][c4] = make_float4(a.x + c.x, a.y + c.y, a.z + c.z, a.w + c.w);
    }
    __syncthreads();
  }
  if (r == 0 && col < len) {
    const float4 v = red[0][c4];
    float4* d = reinterpret_cast<float4*>(dst + col);
    if (accumulate) {
      const float4 o = *d;
      *d = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
    } else {
      *d = v;
    }
  }
}

// Many reductions in one launch: task t sums nblk[t] rows of len[t] floats
// (row stride len[t]) into dst[t]; blocks [start[t], start[t+1]) serve task t
// (the path is uniform per block).
__global__ void __launch_bounds__(1024) slab_reduce_multi_k(SlabTasks T) {
  __shared__ float4 red_v[128][8];
  __shared__ float red_s[16][64];
  int t = 0;
  while (t + 1 < T.ntask && (int)blockIdx.x >= T.start[t + 1]) ++t;
  const int blk = (int)blockIdx.x - T.start[t];
  if (T.vec[t])
    slab_cols_vec(T.src[t], T.dst[t], T.len[t], T.nblk[t], blk, T.accumulate, red_v);
  else
    slab_cols_scalar(T.src[t], T.dst[t], T.len[t], T.nblk[t], blk, T.accumulate, red_s);
}

// part[s][n] = sum over rows r in stripe s of X[r][n]
__global__ void __launch_bounds__(256) colsum_part_k(const float* __restrict__ X, int M, int N, long long ld,
                                                     float* __restrict__ part, int rows_per) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + lane;
  const int r0 = blockIdx.y * rows_per;
  int r1 = r0 + rows_per;
  if (r1 > M) r1 = M;
  float s = 0.f;
  if (n < N)
    for (int r = r0 + wv; r < r1; r += 4) s += X[(long long)r * ld + n];
  red[wv][lane] = s;
  __syncthreads();
  if (wv == 0 && n < N) part[(long long)blockIdx.y * N + n] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

__global__ void axpby_k(const float* __restrict__ x, float* __restrict__ y, long long n, float a, float b) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    y[i] = a * x[i] + (b == 0.f ? 0.f : b * y[i]);
}

// the 32-bit instantiation: the grid-stride step (<= 8192 x 256 threads) must
// not overflow past the last element either
static inline bool int_index_ok(long long n) { return n + 8192LL * 256 < (1ll << 31); }
static inline int grid_for(long long n, int bs = 256) {
  long long g = (n + bs - 1) / bs;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

extern "C" {

int paig_maxpool2_fwd(const float* x, long long x_fs, float* y, long long y_fs, int F, int C, int H, int W,
                      void* stream) {
  if (F <= 0) return 0;
  if (H % 2 == 0 && W % 4 == 0 && x_fs % 4 == 0 && y_fs % 2 == 0 && (long long)F * C * H * W < (1ll << 31) &&
      (uintptr_t)x % 16 == 0 && (uintptr_t)y % 8 == 0) {
    const long long nv = (long long)F * C * (H / 2) * (W / 4);
    hipLaunchKernelGGL(maxpool_fwd_v_k, dim3(grid_for(nv)), dim3(256), 0, (hipStream_t)stream, FView{x, x_fs, 0, 0},
                       FViewW{y, y_fs}, F, C, H, W);
    PAIG_CHECK_LAUNCH();
    return 0;
  }
  long long n = (long long)F * C * (H / 2) * (W / 2);
  if (int_index_ok(n))
    hipLaunchKernelGGL(maxpool_fwd_k<int>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, FView{x, x_fs, 0, 0},
                     FViewW{y, y_fs}, F, C, H, W);
  else
    hipLaunchKernelGGL(maxpool_fwd_k<long long>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, FView{x, x_fs, 0, 0},
                     FViewW{y, y_fs}, F, C, H, W);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_maxpool2_fwd_codes(const float* x, long long x_fs, float* y, long long y_fs, unsigned char* code,
                            long long code_fs, int F, int C, int H, int W, void* stream) {
  if (F <= 0) return 0;
  PAIG_REQUIRE(H % 2 == 0 && W % 2 == 0 && code && code_fs >= (long long)(C + 7) / 8 * 8 * (H / 2) * (W / 2) &&
                   (long long)F * C * H * W < (1ll << 31),
               "paig_maxpool2_fwd_codes: needs even H, W, a code frame of C/8 x H/2 x W/2 x 8 bytes (C=%d H=%d W=%d)",
               C, H, W);
  const long long n = (long long)F * C * (H / 2) * (W / 2);
  hipLaunchKernelGGL(maxpool_fwd_codes_k, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, FView{x, x_fs, 0, 0},
                     FViewW{y, y_fs}, code, code_fs, F, C, H, W);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_maxpool2_bwd_relu(const float* x, long long x_fs, const float* dy, long long dy_fs, float* dx, long long dx_fs,
                           int F, int C, int H, int W, void* stream) {
  if (F <= 0) return 0;
  if (H % 2 == 0 && W % 4 == 0 && x_fs % 4 == 0 && dx_fs % 4 == 0 && dy_fs % 2 == 0 &&
      (long long)F * C * H * W < (1ll << 31) && (uintptr_t)x % 16 == 0 && (uintptr_t)dx % 16 == 0 &&
      (uintptr_t)dy % 8 == 0) {
    const long long nv = (long long)F * C * (H / 2) * (W / 4);
    hipLaunchKernelGGL(maxpool_bwd_relu_v_k, dim3(grid_for(nv)), dim3(256), 0, (hipStream_t)stream,
                       FView{x, x_fs, 0, 0}, FView{dy, dy_fs, 0, 0}, FViewW{dx, dx_fs}, F, C, H, W);
    PAIG_CHECK_LAUNCH();
    return 0;
  }
  long long n = (long long)F * C * H * W;
  if (int_index_ok(n))
    hipLaunchKernelGGL(maxpool_bwd_relu_k<int>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, FView{x, x_fs, 0, 0},
                     FView{dy, dy_fs, 0, 0}, FViewW{dx, dx_fs}, F, C, H, W);
  else
    hipLaunchKernelGGL(maxpool_bwd_relu_k<long long>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, FView{x, x_fs, 0, 0},
                     FView{dy, dy_fs, 0, 0}, FViewW{dx, dx_fs}, F, C, H, W);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_upsample2_fwd(const float* s, long long s_fs, float* u, long long u_fs, int F, int C, int Hs, int Ws, int Ho,
                       int Wo, void* stream) {
  if (F <= 0) return 0;
  long long n = (long long)F * C * Ho * Wo;
  if (int_index_ok(n))
    hipLaunchKernelGGL(upsample_fwd_k<int>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, FView{s, s_fs, 0, 0},
                     FViewW{u, u_fs}, F, C, Hs, Ws, Ho, Wo);
  else
    hipLaunchKernelGGL(upsample_fwd_k<long long>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, FView{s, s_fs, 0, 0},
                     FViewW{u, u_fs}, F, C, Hs, Ws, Ho, Wo);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_upsample2_bwd(const float* du, long long du_fs, const float* s, long long s_fs, float* ds, long long ds_fs,
                       int F, int C, int Hs, int Ws, int Ho, int Wo, int relu_mask, void* stream) {
  if (F <= 0) return 0;
  PAIG_REQUIRE(Ho == 2 * Hs && Wo == 2 * Ws, "upsample_bwd: exact 2x upscale only (Resize(H/2 -> H))");
  if (Ws % 2 == 0 && Wo % 4 == 0 && du_fs % 4 == 0 && ds_fs % 2 == 0 && (!relu_mask || s_fs % 2 == 0) &&
      (long long)F * C * Ho * Wo < (1ll << 31) && (uintptr_t)du % 16 == 0 && (uintptr_t)ds % 8 == 0 &&
      (!relu_mask || (uintptr_t)s % 8 == 0)) {
    const long long nv = (long long)F * C * Hs * (Ws / 2);
    hipLaunchKernelGGL(upsample_bwd_v_k, dim3(grid_for(nv)), dim3(256), 0, (hipStream_t)stream,
                       FView{du, du_fs, 0, 0}, FView{s, s_fs, 0, 0}, FViewW{ds, ds_fs}, F, C, Hs, Ws, relu_mask);
    PAIG_CHECK_LAUNCH();
    return 0;
  }
  long long n = (long long)F * C * Hs * Ws;
  if (int_index_ok(n))
    hipLaunchKernelGGL(upsample_bwd_k<int>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, FView{du, du_fs, 0, 0},
                     FView{s, s_fs, 0, 0}, FViewW{ds, ds_fs}, F, C, Hs, Ws, Ho, Wo, relu_mask);
  else
    hipLaunchKernelGGL(upsample_bwd_k<long long>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, FView{du, du_fs, 0, 0},
                     FView{s, s_fs, 0, 0}, FViewW{ds, ds_fs}, F, C, Hs, Ws, Ho, Wo, relu_mask);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_mask_softmax_fwd(const float* logits, const float* x, long long x_fs, int x_grp, long long x_gs,
                          float* masks, float* objs, float* pobjs, int F, int K, int C, int H, int W, void* stream) {
  if (F <= 0) return 0;
  PAIG_REQUIRE(K >= 1 && K <= 7, "mask_softmax: K=%d", K);
  if (pobjs) {
    PAIG_REQUIRE(C <= 3 && H % 2 == 0 && W % 2 == 0, "mask_softmax pooled: C=%d H=%d W=%d", C, H, W);
    hipLaunchKernelGGL(mask_softmax_pool_fwd_k, dim3(grid_for((long long)F * (H / 2) * (W / 2))), dim3(256), 0,
                       (hipStream_t)stream, logits, FView{x, x_fs, x_gs, x_grp}, masks, objs, pobjs, F, K, C, H, W);
  } else {
    const bool v4 = (H * W) % 4 == 0 && C <= 3 && (K == 2 || K == 3) && x_fs % 4 == 0 && x_gs % 4 == 0 &&
                    ((uintptr_t)logits | (uintptr_t)x | (uintptr_t)masks | (uintptr_t)objs) % 16 == 0;
    const dim3 g4(grid_for((long long)F * H * W / 4));
    if (v4 && K == 2)
      hipLaunchKernelGGL(mask_softmax_fwd_v_k<2>, g4, dim3(256), 0, (hipStream_t)stream, logits,
                         FView{x, x_fs, x_gs, x_grp}, masks, objs, F, C, H * W);
    else if (v4 && K == 3)
      hipLaunchKernelGGL(mask_softmax_fwd_v_k<3>, g4, dim3(256), 0, (hipStream_t)stream, logits,
                         FView{x, x_fs, x_gs, x_grp}, masks, objs, F, C, H * W);
    else
      hipLaunchKernelGGL(mask_softmax_fwd_k, dim3(grid_for((long long)F * H * W)), dim3(256), 0, (hipStream_t)stream,
                         logits, FView{x, x_fs, x_gs, x_grp}, masks, objs, F, K, C, H * W);
  }
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_mask_softmax_bwd(const float* logits, const float* x, long long x_fs, int x_grp, long long x_gs,
                          const float* masks, const float* dobjs, float* dlogits, int F, int K, int C, int H, int W,
                          int flags, void* stream) {
  if (F <= 0) return 0;
  PAIG_REQUIRE(K >= 1 && K <= 7, "mask_softmax: K=%d", K);
  const bool v4 = !(flags & 2) && (H * W) % 4 == 0 && C <= 3 && (K == 2 || K == 3) && x_fs % 4 == 0 &&
                  x_gs % 4 == 0 &&
                  ((uintptr_t)logits | (uintptr_t)x | (uintptr_t)masks | (uintptr_t)dobjs | (uintptr_t)dlogits) % 16 == 0;
  const dim3 g4(grid_for((long long)F * H * W / 4));
  if (v4 && K == 2)
    hipLaunchKernelGGL(mask_softmax_bwd_v_k<2>, g4, dim3(256), 0, (hipStream_t)stream, logits,
                       FView{x, x_fs, x_gs, x_grp}, masks, dobjs, dlogits, F, C, H * W, flags);
  else if (v4 && K == 3)
    hipLaunchKernelGGL(mask_softmax_bwd_v_k<3>, g4, dim3(256), 0, (hipStream_t)stream, logits,
                       FView{x, x_fs, x_gs, x_grp}, masks, dobjs, dlogits, F, C, H * W, flags);
  else
    hipLaunchKernelGGL(mask_softmax_bwd_k, dim3(grid_for((long long)F * H * W)), dim3(256), 0, (hipStream_t)stream,
                       logits, FView{x, x_fs, x_gs, x_grp}, masks, dobjs, dlogits, F, K, C, H, W, flags);
  PAIG_CHECK_LAUNCH();
  return 0;
}

static bool head_mask_ok(const void* a, const void* b, const void* c, const void* d, const void* e, long long x_fs,
                         long long x_gs, int K, int H, int W) {
  return (H * W) % 4 == 0 && (K == 2 || K == 3) && x_fs % 4 == 0 && x_gs % 4 == 0 &&
         ((uintptr_t)a | (uintptr_t)b | (uintptr_t)c | (uintptr_t)d | (uintptr_t)e) % 16 == 0;
}
// the two heads: ShallowUNet (CI 8, ReLU'd logits: flags 1), UNet (CI 16,
// pooled objects: flags 2)
static bool head_mask_kind(int CI, int flags, int H, int W, const void* pobjs) {
  if (CI == 8 && flags == 1) return true;
  return CI == 16 && flags == 2 && H % 2 == 0 && W % 4 == 0 && ((uintptr_t)pobjs % 8) == 0;
}

int paig_head_mask_blocks(int F, int H, int W) {
  const long long n = (long long)F * H * W / 4;
  long long g = (n + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 1024 ? 1024 : g));
}

int paig_head_mask_fwd_ex(const float* xl, const float* w, const float* b, const float* x, long long x_fs, int x_grp,
                          long long x_gs, float* masks, float* objs, float* pobjs, int F, int K, int CI, int H, int W,
                          int flags, void* stream) {
  if (F <= 0) return 0;
  PAIG_REQUIRE(head_mask_ok(xl, x, masks, objs, nullptr, x_fs, x_gs, K, H, W),
               "head_mask_fwd: needs K in {2,3}, H*W %% 4 == 0 and 16-byte aligned buffers (K=%d H=%d W=%d)", K, H, W);
  PAIG_REQUIRE(head_mask_kind(CI, flags, H, W, pobjs) && (!(flags & 2) || pobjs),
               "head_mask_fwd: (CI=%d, flags=%d) is neither the ShallowUNet head (8, 1) nor the UNet's (16, 2)", CI,
               flags);
  const FView xv{x, x_fs, x_gs, x_grp};
  hipStream_t st = (hipStream_t)stream;
  if (flags & 2) {
    const dim3 g(grid_for((long long)F * (H / 2) * (W / 4)));
    if (K == 2) hipLaunchKernelGGL((head_mask_pool_fwd_k<2, 16, false>), g, dim3(256), 0, st, xl, w, b, xv, masks, objs, pobjs, F, H, W);
    else hipLaunchKernelGGL((head_mask_pool_fwd_k<3, 16, false>), g, dim3(256), 0, st, xl, w, b, xv, masks, objs, pobjs, F, H, W);
  } else {
    const dim3 g(grid_for((long long)F * H * W / 4));
    if (K == 2) hipLaunchKernelGGL((head_mask_fwd_k<2, 8, true>), g, dim3(256), 0, st, xl, w, b, xv, masks, objs, F, H * W);
    else hipLaunchKernelGGL((head_mask_fwd_k<3, 8, true>), g, dim3(256), 0, st, xl, w, b, xv, masks, objs, F, H * W);
  }
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_head_mask_bwd_ex(const float* xl, const float* w, const float* b, const float* x, long long x_fs, int x_grp,
                          long long x_gs, const float* masks, const float* dobjs, float* dxl, float* slab, int F, int K,
                          int CI, int H, int W, int flags, void* stream) {
  if (F <= 0) return 0;
  PAIG_REQUIRE(head_mask_ok(xl, x, masks, (flags & 2) ? nullptr : dobjs, dxl, x_fs, x_gs, K, H, W),
               "head_mask_bwd: needs K in {2,3}, H*W %% 4 == 0 and 16-byte aligned buffers (K=%d H=%d W=%d)", K, H, W);
  PAIG_REQUIRE(head_mask_kind(CI, flags, H, W, dobjs),
               "head_mask_bwd: (CI=%d, flags=%d) is neither the ShallowUNet head (8, 1) nor the UNet's (16, 2)", CI,
               flags);
  const dim3 g(paig_head_mask_blocks(F, H, W));
  const FView xv{x, x_fs, x_gs, x_grp};
  hipStream_t st = (hipStream_t)stream;
  if (flags & 2) {
    if (K == 2) hipLaunchKernelGGL((head_mask_bwd_k<2, 16, false, true>), g, dim3(256), 0, st, xl, w, b, xv, masks, dobjs, dxl, slab, F, H, W);
    else hipLaunchKernelGGL((head_mask_bwd_k<3, 16, false, true>), g, dim3(256), 0, st, xl, w, b, xv, masks, dobjs, dxl, slab, F, H, W);
  } else {
    if (K == 2) hipLaunchKernelGGL((head_mask_bwd_k<2, 8, true, false>), g, dim3(256), 0, st, xl, w, b, xv, masks, dobjs, dxl, slab, F, H, W);
    else hipLaunchKernelGGL((head_mask_bwd_k<3, 8, true, false>), g, dim3(256), 0, st, xl, w, b, xv, masks, dobjs, dxl, slab, F, H, W);
  }
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_head_mask_fwd(const float* x12, const float* w, const float* b, const float* x, long long x_fs, int x_grp,
                       long long x_gs, float* masks, float* objs, int F, int K, int H, int W, void* stream) {
  return paig_head_mask_fwd_ex(x12, w, b, x, x_fs, x_grp, x_gs, masks, objs, nullptr, F, K, 8, H, W, 1, stream);
}

int paig_head_mask_bwd(const float* x12, const float* w, const float* b, const float* x, long long x_fs, int x_grp,
                       long long x_gs, const float* masks, const float* dobjs, float* dx12, float* slab, int F, int K,
                       int H, int W, void* stream) {
  return paig_head_mask_bwd_ex(x12, w, b, x, x_fs, x_grp, x_gs, masks, dobjs, dx12, slab, F, K, 8, H, W, 1, stream);
}

int paig_pos_head_fwd(const float* h3, float* pos, int N, int K, float half, void* stream) {
  hipLaunchKernelGGL(pos_head_fwd_k, dim3(grid_for(N * K * 2)), dim3(256), 0, (hipStream_t)stream, h3, pos, N, K, half);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_pos_head_bwd(const float* h3, const float* dpos, float* dh3, int N, int K, float half, void* stream) {
  hipLaunchKernelGGL(pos_head_bwd_k, dim3(grid_for(N * K * 2)), dim3(256), 0, (hipStream_t)stream, h3, dpos, dh3, N, K,
                     half);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_vel_pack(const float* pos, float* X, int B, int Te, int K, int S, int alt, void* stream) {
  hipLaunchKernelGGL(vel_pack_k, dim3(grid_for(K * B * S * 2)), dim3(256), 0, (hipStream_t)stream, pos, X, B, Te, K, S,
                     alt);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_vel_unpack_add(const float* dX, const float* dpos0, float* dpos, int B, int Te, int K, int S, int alt,
                        void* stream) {
  hipLaunchKernelGGL(vel_unpack_add_k, dim3(grid_for(B * S * 2 * K)), dim3(256), 0, (hipStream_t)stream, dX, dpos0,
                     dpos, B, Te, K, S, alt);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_slab_reduce_multi(int ntask, const float* const* src, const int* nblk, const int* len, float* const* dst,
                           int accumulate, void* stream) {
  PAIG_REQUIRE(ntask >= 0 && ntask <= PAIG_MAX_SLAB_TASKS, "slab_reduce_multi: %d tasks", ntask);
  if (ntask == 0) return 0;
  SlabTasks T;
  int blocks = 0;
  for (int t = 0; t < ntask; ++t) {
    PAIG_REQUIRE(len[t] >= 0 && nblk[t] >= 0, "slab_reduce_multi: task %d len %d nblk %d", t, len[t], nblk[t]);
    T.src[t] = src[t];
    T.dst[t] = dst[t];
    T.nblk[t] = nblk[t];
    T.len[t] = len[t];
    T.vec[t] = len[t] % 4 == 0 && ((uintptr_t)src[t] & 15) == 0 && ((uintptr_t)dst[t] & 15) == 0;
    T.start[t] = blocks;
    blocks += cdiv(len[t], T.vec[t] ? 32 : 64);
  }
  T.start[ntask] = blocks;
  T.ntask = ntask;
  T.accumulate = accumulate;
  if (blocks == 0) return 0;
  hipLaunchKernelGGL(slab_reduce_multi_k, dim3(blocks), dim3(1024), 0, (hipStream_t)stream, T);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_slab_reduce(const float* slab, int nblk, long long ld, int len, float* out, int accumulate, void* stream) {
  if (len <= 0) return 0;
  hipLaunchKernelGGL(slab_reduce_k, dim3(cdiv(len, 64)), dim3(256), 0, (hipStream_t)stream, slab, nblk, ld, len, out,
                     accumulate);
  PAIG_CHECK_LAUNCH();
  return 0;
}

// out[n] (+)= sum_r X[r][n]; workspace >= stripes*N floats (stripes = ceil(M/rows_per)).
size_t paig_colsum_workspace(int M, int N) {
  int rows_per = 256;
  int stripes = cdiv(M, rows_per);
  return (size_t)stripes * N;
}

int paig_colsum(const float* X, int M, int N, long long ld, float* out, int accumulate, float* ws, void* stream) {
  if (N <= 0) return 0;
  int rows_per = 256;
  int stripes = cdiv(M, rows_per);
  if (M <= 0) {
    stripes = 0;
  } else {
    hipLaunchKernelGGL(colsum_part_k, dim3(cdiv(N, 64), stripes), dim3(256), 0, (hipStream_t)stream, X, M, N, ld, ws,
                       rows_per);
    PAIG_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(slab_reduce_k, dim3(cdiv(N, 64)), dim3(256), 0, (hipStream_t)stream, ws, stripes, (long long)N, N,
                     out, accumulate);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_axpby(const float* x, float* y, long long n, float a, float b, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(axpby_k, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, y, n, a, b);
  PAIG_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
