// U-Net 3x3 / 1x1 "same" convolutions for the PhysicsNet encoder
// (reference: nn/network/blocks.py:113-170 UNet, :246-276 ShallowUNet, run by
// aten conv2d in the reference).
//
// Design (CDNA4, fp32):
//  * direct convolution on the VALU: each thread owns PX=4 horizontally
//    adjacent output pixels x CO(<=8) output channels (32 accumulators);
//  * the input tile (frames x rows + halo, one 8-channel chunk at a time) is
//    staged in LDS with an odd row pitch (ds_read_b32 bank spread);
//  * weights are wave-uniform (the output-channel group is fixed per wave via
//    readfirstlane), so hipcc fetches them with scalar loads into SGPRs and
//    every v_fma takes one SGPR operand: no LDS/VGPR traffic for weights;
//  * dgrad is the same kernel with the weight indexed transposed + flipped,
//    and an epilogue that applies the ReLU derivative of the layer input;
//  * wgrad reduces dY (x) im2col(X) over pixels per thread, over the block's
//    pixel partitions by wave shuffles, and over blocks through a partial slab
//    (deterministic, no atomics) summed by paig_slab_reduce.
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

namespace {

constexpr int PX = 4;
constexpr int FL_RELU = 1;   // out = max(out, 0)
constexpr int FL_MASK = 2;   // out *= (aux > 0)       (ReLU'(layer input))
constexpr int FL_ACCUM = 4;  // out += existing value

template <int CIN, int COUT, int CO, int KS, bool DGRAD>
__global__ void __launch_bounds__(256)
conv_fwd_k(FView in, FViewW out, FView aux, const float* __restrict__ w, const float* __restrict__ bias,
           int F, int H, int W, int FPB, int RPB, int GB, int flags) {
  constexpr int HALO = KS - 1, PADL = KS / 2, KK = KS * KS;
  constexpr int CIC = CIN < 8 ? CIN : 8;
  static_assert(CIN % CIC == 0, "CIN must be a multiple of the chunk");
  constexpr int NCHUNK = CIN / CIC;
  extern __shared__ __attribute__((aligned(16))) float lds[];

  const int CGR = (W + PX - 1) / PX;
  const int TW = CGR * PX + HALO;
  const int TWP = TW | 1;
  const int TR = RPB + HALO;
  const int nthreads = blockDim.x;
  const int SLOTS = nthreads / GB;
  const int tid = threadIdx.x;
  const int cog = uniform_i(blockIdx.y * GB + tid / SLOTS);
  const int slot = tid % SLOTS;
  const int nRB = (H + RPB - 1) / RPB;
  const int fb = blockIdx.x / nRB, rb = blockIdx.x % nRB;
  const int f0 = fb * FPB, y0 = rb * RPB;
  const int per_frame = RPB * CGR;
  const int fi = slot / per_frame;
  const int rem = slot % per_frame;
  const int r = rem / CGR, cg = rem % CGR;
  const int f = f0 + fi, y = y0 + r, x0 = cg * PX;
  const bool valid = (fi < FPB) && (f < F) && (y < H) && (r < RPB);

  float acc[CO][PX];
#pragma unroll
  for (int co = 0; co < CO; ++co)
#pragma unroll
    for (int p = 0; p < PX; ++p) acc[co][p] = 0.f;

  const int E = FPB * CIC * TR * TW;
  for (int ch = 0; ch < NCHUNK; ++ch) {
    const int ci0 = ch * CIC;
    for (int i = tid; i < E; i += nthreads) {
      int cc = i % TW;
      int t = i / TW;
      int rr = t % TR;
      t /= TR;
      int c = t % CIC;
      int ff = t / CIC;
      int gf = f0 + ff, gy = y0 + rr - PADL, gx = cc - PADL;
      float v = 0.f;
      if (gf < F && gy >= 0 && gy < H && gx >= 0 && gx < W) v = in.frame(gf)[((ci0 + c) * H + gy) * W + gx];
      lds[((ff * CIC + c) * TR + rr) * TWP + cc] = v;
    }
    __syncthreads();
    if (valid) {
      const float* base = lds + (fi * CIC * TR + r) * TWP + x0;
#pragma unroll
      for (int c = 0; c < CIC; ++c) {
        float win[KS][PX + KS - 1];
#pragma unroll
        for (int ky = 0; ky < KS; ++ky)
#pragma unroll
          for (int j = 0; j < PX + KS - 1; ++j) win[ky][j] = base[(c * TR + ky) * TWP + j];
#pragma unroll
        for (int co = 0; co < CO; ++co) {
          const int cg_o = cog * CO + co;
#pragma unroll
          for (int ky = 0; ky < KS; ++ky)
#pragma unroll
            for (int kx = 0; kx < KS; ++kx) {
              float wv;
              if (DGRAD)
                wv = w[((ci0 + c) * COUT + cg_o) * KK + (KS - 1 - ky) * KS + (KS - 1 - kx)];
              else
                wv = w[(cg_o * CIN + ci0 + c) * KK + ky * KS + kx];
#pragma unroll
              for (int p = 0; p < PX; ++p) acc[co][p] = fmaf(wv, win[ky][p + kx], acc[co][p]);
            }
        }
      }
    }
    __syncthreads();
  }

  if (!valid) return;
  const long long HW = (long long)H * W;
  float* op = out.frame(f) + (long long)(cog * CO) * HW + (long long)y * W + x0;
  const float* ap = (flags & FL_MASK) ? aux.frame(f) + (long long)(cog * CO) * HW + (long long)y * W + x0 : nullptr;
#pragma unroll
  for (int co = 0; co < CO; ++co) {
    const float b = bias ? bias[cog * CO + co] : 0.f;
#pragma unroll
    for (int p = 0; p < PX; ++p) {
      if (x0 + p < W) {
        float v = acc[co][p] + b;
        if (flags & FL_RELU) v = v < 0.f ? 0.f : v;
        if (flags & FL_ACCUM) v += op[co * HW + p];
        if (flags & FL_MASK) v = ap[co * HW + p] > 0.f ? v : 0.f;
        op[co * HW + p] = v;
      }
    }
  }
}

template <int CIN, int COUT, int CO, int KS>
__global__ void __launch_bounds__(256)
conv_wgrad_k(FView x, FView dy, float* __restrict__ slab, int F, int H, int W, int FPB, int RPB, int PP,
             int ntiles) {
  constexpr int HALO = KS - 1, PADL = KS / 2, KK = KS * KS;
  constexpr int NCOB = COUT / CO;
  static_assert(COUT % CO == 0, "COUT % CO");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int CGR = (W + PX - 1) / PX;
  const int DW = CGR * PX;
  const int TW = DW + HALO;
  const int TWP = TW | 1;
  const int TR = RPB + HALO;
  const int tid = threadIdx.x;
  const int nthreads = blockDim.x;
  // (cout group, ci) combos: blockIdx.y selects this block's slice of them
  const int combo = blockIdx.y * (nthreads / PP) + tid / PP, pp = tid % PP;
  const int cob = combo / CIN, ci = combo % CIN;
  float* xs = lds;
  float* ds = lds + FPB * CIN * TR * TWP;

  float acc[CO][KK];
  float bacc[CO];
#pragma unroll
  for (int co = 0; co < CO; ++co) {
    bacc[co] = 0.f;
#pragma unroll
    for (int k = 0; k < KK; ++k) acc[co][k] = 0.f;
  }

  const int nRB = (H + RPB - 1) / RPB;
  const int EX = FPB * CIN * TR * TW;
  const int ED = FPB * COUT * RPB * DW;
  const int ngroups = FPB * RPB * CGR;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int fb = tile / nRB, rb = tile % nRB;
    const int f0 = fb * FPB, y0 = rb * RPB;
    for (int i = tid; i < EX; i += nthreads) {
      int cc = i % TW;
      int t = i / TW;
      int rr = t % TR;
      t /= TR;
      int c = t % CIN;
      int ff = t / CIN;
      int gf = f0 + ff, gy = y0 + rr - PADL, gx = cc - PADL;
      float v = 0.f;
      if (gf < F && gy >= 0 && gy < H && gx >= 0 && gx < W) v = x.frame(gf)[(c * H + gy) * W + gx];
      xs[((ff * CIN + c) * TR + rr) * TWP + cc] = v;
    }
    for (int i = tid; i < ED; i += nthreads) {
      int cc = i % DW;
      int t = i / DW;
      int rr = t % RPB;
      t /= RPB;
      int c = t % COUT;
      int ff = t / COUT;
      int gf = f0 + ff, gy = y0 + rr;
      float v = 0.f;
      if (gf < F && gy < H && cc < W) v = dy.frame(gf)[(c * H + gy) * W + cc];
      ds[i] = v;
    }
    __syncthreads();
    for (int g = pp; g < ngroups; g += PP) {
      const int fi = g / (RPB * CGR);
      const int rem = g % (RPB * CGR);
      const int r = rem / CGR, cg = rem % CGR;
      const float* xb = xs + ((fi * CIN + ci) * TR + r) * TWP + cg * PX;
      const float* db = ds + ((fi * COUT + cob * CO) * RPB + r) * DW + cg * PX;
      float win[KS][PX + KS - 1];
#pragma unroll
      for (int ky = 0; ky < KS; ++ky)
#pragma unroll
        for (int j = 0; j < PX + KS - 1; ++j) win[ky][j] = xb[ky * TWP + j];
#pragma unroll
      for (int co = 0; co < CO; ++co) {
        float d[PX];
#pragma unroll
        for (int p = 0; p < PX; ++p) d[p] = db[co * RPB * DW + p];
#pragma unroll
        for (int p = 0; p < PX; ++p) bacc[co] += d[p];
#pragma unroll
        for (int ky = 0; ky < KS; ++ky)
#pragma unroll
          for (int kx = 0; kx < KS; ++kx)
#pragma unroll
            for (int p = 0; p < PX; ++p) acc[co][ky * KS + kx] = fmaf(d[p], win[ky][p + kx], acc[co][ky * KS + kx]);
      }
    }
    __syncthreads();
  }

  // reduce over the PP lanes of a combo (adjacent lanes, PP | 64, power of 2)
#pragma unroll
  for (int co = 0; co < CO; ++co) {
#pragma unroll
    for (int k = 0; k < KK; ++k) {
      float v = acc[co][k];
      for (int o = PP >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      acc[co][k] = v;
    }
    float v = bacc[co];
    for (int o = PP >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    bacc[co] = v;
  }
  if (pp == 0) {
    float* s = slab + (long long)blockIdx.x * (COUT * CIN * KK + COUT);
#pragma unroll
    for (int co = 0; co < CO; ++co) {
#pragma unroll
      for (int k = 0; k < KK; ++k) s[((cob * CO + co) * CIN + ci) * KK + k] = acc[co][k];
      if (ci == 0) s[COUT * CIN * KK + cob * CO + co] = bacc[co];
    }
  }
  (void)NCOB;
}

// ---- host-side dispatch -----------------------------------------------------

struct FwdGeom {
  int FPB, RPB, GB, G, threads, lds_bytes;
  dim3 grid;
};

static FwdGeom fwd_geom(int F, int H, int W, int CIN, int COUT, int CO, int KS) {
  FwdGeom g;
  const int CIC = CIN < 8 ? CIN : 8;
  g.G = COUT / CO;
  g.GB = g.G % 4 == 0 ? 4 : (g.G % 2 == 0 ? 2 : 1);   // cout groups per block: a divisor of G
  int target = (256 / g.GB) / 64 * 64;  // slots per cout group (multiple of 64)
  if (target < 64) target = 64;
  const int CGR = (W + PX - 1) / PX;
  const int per_frame = H * CGR;
  if (per_frame >= target) {
    g.FPB = 1;
    g.RPB = target / CGR;
    if (g.RPB < 1) g.RPB = 1;
    if (g.RPB > H) g.RPB = H;
  } else {
    g.FPB = target / per_frame;
    g.RPB = H;
  }
  int slots = g.FPB * g.RPB * CGR;
  slots = (slots + 63) / 64 * 64;
  g.threads = slots * g.GB;
  const int TW = CGR * PX + KS - 1;
  const int TWP = TW | 1;
  g.lds_bytes = g.FPB * CIC * (g.RPB + KS - 1) * TWP * 4;
  const int nRB = (H + g.RPB - 1) / g.RPB;
  g.grid = dim3((unsigned)(cdiv(F, g.FPB) * nRB), (unsigned)(g.G / g.GB), 1);
  return g;
}

template <int CIN, int COUT, int KS, bool DG>
static int launch_fwd(FView in, FViewW out, FView aux, const float* w, const float* b, int F, int H, int W,
                      int flags, hipStream_t st) {
  constexpr int CO = COUT < 8 ? COUT : 8;
  FwdGeom g = fwd_geom(F, H, W, CIN, COUT, CO, KS);
  if (g.G % g.GB != 0) {
    paig_set_error("conv: cout groups %d not a multiple of %d", g.G, g.GB);
    return PAIG_E_UNSUPPORTED;
  }
  if (g.threads > 256 || g.lds_bytes > 64 * 1024) {   // __launch_bounds__(256)
    paig_set_error("conv: geometry too large (threads %d, lds %d)", g.threads, g.lds_bytes);
    return PAIG_E_UNSUPPORTED;
  }
  hipLaunchKernelGGL((conv_fwd_k<CIN, COUT, CO, KS, DG>), g.grid, dim3(g.threads), g.lds_bytes, st, in, out, aux,
                     w, b, F, H, W, g.FPB, g.RPB, g.GB, flags);
  PAIG_CHECK_LAUNCH();
  return 0;
}

template <int CIN, int COUT, int KS>
static int launch_wgrad(FView x, FView dy, float* slab, int nblk_max, int* nblk_out, int F, int H, int W,
                        hipStream_t st) {
  constexpr int CO = COUT < 8 ? COUT : 8;
  constexpr int NCOMBO = (COUT / CO) * CIN;
  int PP = 1;
  while (PP * 2 * NCOMBO <= 256 && PP < 64) PP *= 2;
  // more combos than one 256-thread block holds (UNet): split them over gridDim.y
  int CPB = NCOMBO, GY = 1;
  while (CPB * PP > 256 && CPB % 2 == 0) {
    CPB /= 2;
    GY *= 2;
  }
  const int threads = CPB * PP;
  if (threads > 256 || threads % 64 != 0) {
    paig_set_error("wgrad: %d combos cannot be split into blocks", NCOMBO);
    return PAIG_E_UNSUPPORTED;
  }
  const int CGR = (W + PX - 1) / PX;
  const int DW = CGR * PX;
  const int TWP = (DW + KS - 1) | 1;
  auto lds_of = [&](int fpb, int rpb) { return 4 * fpb * (CIN * (rpb + KS - 1) * TWP + COUT * rpb * DW); };
  int FPB = 1, RPB = H;
  while (RPB > 1 && lds_of(1, RPB) > 48 * 1024) RPB = (RPB + 1) / 2;
  if (RPB == H)
    while (FPB < 16 && lds_of(FPB * 2, RPB) <= 32 * 1024 && FPB * 2 <= F) FPB *= 2;
  const int lds = lds_of(FPB, RPB);
  const int nRB = (H + RPB - 1) / RPB;
  const int ntiles = cdiv(F, FPB) * nRB;
  int nblk = ntiles < nblk_max ? ntiles : nblk_max;
  if (nblk < 1) nblk = 1;
  *nblk_out = nblk;
  hipLaunchKernelGGL((conv_wgrad_k<CIN, COUT, CO, KS>), dim3(nblk, GY), dim3(threads), lds, st, x, dy, slab, F, H, W,
                     FPB, RPB, PP, ntiles);
  PAIG_CHECK_LAUNCH();
  return 0;
}

// (CIN, COUT, KS) combinations used by ShallowUNet(hidden 8) and UNet(hidden 16)
// in forward, and their transposes in dgrad.
#define PAIG_CONV_SHAPES(X)                                                                          \
  X(3, 8, 3) X(8, 8, 3) X(8, 16, 3) X(16, 16, 3) X(16, 32, 3) X(32, 32, 3) X(32, 16, 3) X(24, 8, 3) \
  X(8, 2, 1) X(16, 8, 3) X(8, 24, 3) X(2, 8, 1) X(3, 16, 3) X(32, 64, 3) X(64, 64, 3) X(64, 128, 3) \
  X(128, 128, 3) X(128, 32, 3) X(96, 64, 3) X(64, 32, 3) X(48, 16, 3) X(16, 2, 1) X(2, 16, 1)       \
  X(64, 96, 3) X(16, 48, 3) X(32, 128, 3) X(128, 64, 3) X(64, 16, 3) X(8, 3, 3) X(16, 3, 3)    \
  X(8, 3, 1) X(3, 8, 1) X(16, 3, 1) X(3, 16, 1)

}  // namespace

extern "C" {

// out[f][co_off..] = conv(in) (+bias) (ReLU)      (forward)
// out = conv_transpose-as-dgrad(in = dY) (* aux>0) (dgrad, flags & 8)
// Views: p/fs/grp/gs per frame_view; channel offsets are folded into pointers.
int paig_conv2d_fwd_ex(const float* in, long long in_fs, int in_grp, long long in_gs, float* out, long long out_fs,
                       const float* aux, long long aux_fs, const float* w, const float* bias, int F, int Cin,
                       int Cout, int H, int W, int ks, int flags, float* xmax, int xmax_n, void* stream);

int paig_conv2d_fwd_pw(const float* in, long long in_fs, int in_grp, long long in_gs, float* out, long long out_fs,
                       const float* aux, long long aux_fs, const float* w, const float* bias, int F, int Cin,
                       int Cout, int H, int W, int ks, int flags, float* xmax, int xmax_n, float* pool_out,
                       long long pool_fs, const void* wprep, void* stream);

int paig_conv2d_fwd(const float* in, long long in_fs, int in_grp, long long in_gs, float* out, long long out_fs,
                    const float* aux, long long aux_fs, const float* w, const float* bias, int F, int Cin,
                    int Cout, int H, int W, int ks, int flags, void* stream) {
  return paig_conv2d_fwd_pw(in, in_fs, in_grp, in_gs, out, out_fs, aux, aux_fs, w, bias, F, Cin, Cout, H, W, ks, flags,
                            nullptr, 0, nullptr, 0, nullptr, stream);
}

int paig_conv2d_fwd_ex(const float* in, long long in_fs, int in_grp, long long in_gs, float* out, long long out_fs,
                       const float* aux, long long aux_fs, const float* w, const float* bias, int F, int Cin,
                       int Cout, int H, int W, int ks, int flags, float* xmax, int xmax_n, void* stream) {
  return paig_conv2d_fwd_pw(in, in_fs, in_grp, in_gs, out, out_fs, aux, aux_fs, w, bias, F, Cin, Cout, H, W, ks, flags,
                            xmax, xmax_n, nullptr, 0, nullptr, stream);
}

int paig_conv2d_fwd_pw(const float* in, long long in_fs, int in_grp, long long in_gs, float* out, long long out_fs,
                       const float* aux, long long aux_fs, const float* w, const float* bias, int F, int Cin,
                       int Cout, int H, int W, int ks, int flags, float* xmax, int xmax_n, float* pool_out,
                       long long pool_fs, const void* wprep, void* stream) {
  return paig_conv2d_fwd_pwc(in, in_fs, in_grp, in_gs, out, out_fs, aux, aux_fs, w, bias, F, Cin, Cout, H, W, ks, flags,
                             xmax, xmax_n, pool_out, pool_fs, nullptr, 0, wprep, stream);
}

int paig_conv2d_fwd_pwc(const float* in, long long in_fs, int in_grp, long long in_gs, float* out, long long out_fs,
                        const float* aux, long long aux_fs, const float* w, const float* bias, int F, int Cin,
                        int Cout, int H, int W, int ks, int flags, float* xmax, int xmax_n, float* pool_out,
                        long long pool_fs, unsigned char* pool_code, long long pool_code_fs, const void* wprep,
                        void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (pool_code && !(flags & 64)) {
    paig_set_error("paig_conv2d_fwd_pwc: window codes need the fused pool (flags & 64)");
    return PAIG_E_SHAPE;
  }
  FView vin{in, in_fs, in_gs, in_grp};
  FViewW vout{out, out_fs};
  FView vaux{aux, aux_fs, 0, 0};
  const bool dgrad = (flags & 8) != 0;
  const int fl = flags & 7;
  if (F <= 0) return 0;
  int rc = 0;
  if (flags & 512) {   // dgrad with the transposed-upsample epilogue: split path only
    if (!(flags & 16) && paig_conv_split_fwd(vin, vout, vaux, w, bias, F, Cin, Cout, H, W, ks, flags, st, &rc,
                                             XMax{xmax, xmax_n}, wprep, PoolOut{pool_out, pool_fs, pool_code,
                                                                                 pool_code_fs}))
      return rc;
    paig_set_error("paig_conv2d_fwd: no transposed-upsample dgrad (flags & 512) for Cin=%d Cout=%d H=%d flags=%d", Cin,
                   Cout, H, flags);
    return PAIG_E_UNSUPPORTED;
  }
  if ((flags & 64) && (flags & 16)) {
    paig_set_error("paig_conv2d_fwd: the fused pool (flags & 64) needs the split path");
    return PAIG_E_UNSUPPORTED;
  }
  if (!(flags & 16) &&
      paig_conv_mfma_fwd(vin, vout, vaux, w, bias, F, Cin, Cout, H, W, ks, flags, st, &rc, XMax{xmax, xmax_n}, wprep,
                         PoolOut{pool_out, pool_fs, pool_code, pool_code_fs}))
    return rc;
  if (flags & 32) {
    paig_set_error("paig_conv2d_fwd: fused-upsample input has no instantiation for Cin=%d Cout=%d H=%d", Cin, Cout, H);
    return PAIG_E_UNSUPPORTED;
  }
#define PAIG_CASE(CI, CO, K)                                                                   \
  if (Cin == CI && Cout == CO && ks == K) {                                                   \
    return dgrad ? launch_fwd<CI, CO, K, true>(vin, vout, vaux, w, bias, F, H, W, fl, st)     \
                 : launch_fwd<CI, CO, K, false>(vin, vout, vaux, w, bias, F, H, W, fl, st);   \
  }
  PAIG_CONV_SHAPES(PAIG_CASE)
#undef PAIG_CASE
  paig_set_error("paig_conv2d_fwd: unsupported shape Cin=%d Cout=%d ks=%d", Cin, Cout, ks);
  return PAIG_E_UNSUPPORTED;
}

// Per-block partial weight+bias gradients: slab[nblk][Cout*Cin*ks*ks + Cout].
// *nblk_out receives the number of partial rows written (<= nblk_max).
int paig_conv2d_wgrad_ex(const float* x, long long x_fs, int x_grp, long long x_gs, const float* dy, long long dy_fs,
                         float* slab, int nblk_max, int* nblk_out, int F, int Cin, int Cout, int H, int W, int ks,
                         int flags, const float* xmax, int xmax_n, void* stream);

int paig_conv2d_wgrad(const float* x, long long x_fs, int x_grp, long long x_gs, const float* dy, long long dy_fs,
                      float* slab, int nblk_max, int* nblk_out, int F, int Cin, int Cout, int H, int W, int ks,
                      int flags, void* stream) {
  return paig_conv2d_wgrad_ex(x, x_fs, x_grp, x_gs, dy, dy_fs, slab, nblk_max, nblk_out, F, Cin, Cout, H, W, ks, flags,
                              nullptr, 0, stream);
}

int paig_conv2d_wgrad_ex(const float* x, long long x_fs, int x_grp, long long x_gs, const float* dy, long long dy_fs,
                         float* slab, int nblk_max, int* nblk_out, int F, int Cin, int Cout, int H, int W, int ks,
                         int flags, const float* xmax, int xmax_n, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  FView vx{x, x_fs, x_gs, x_grp};
  FView vd{dy, dy_fs, 0, 0};
  *nblk_out = 0;
  if (F <= 0) return 0;
  int rc = 0;
  if (!(flags & 16) && paig_conv_mfma_wgrad(vx, vd, slab, nblk_max, nblk_out, F, Cin, Cout, H, W, ks, flags, st, &rc,
                                             XMax{const_cast<float*>(xmax), xmax_n}))
    return rc;
  if (flags & 32) {
    paig_set_error("paig_conv2d_wgrad: fused-upsample input has no instantiation for Cin=%d Cout=%d H=%d", Cin, Cout, H);
    return PAIG_E_UNSUPPORTED;
  }
#define PAIG_CASE(CI, CO, K) \
  if (Cin == CI && Cout == CO && ks == K) return launch_wgrad<CI, CO, K>(vx, vd, slab, nblk_max, nblk_out, F, H, W, st);
  PAIG_CONV_SHAPES(PAIG_CASE)
#undef PAIG_CASE
  paig_set_error("paig_conv2d_wgrad: unsupported shape Cin=%d Cout=%d ks=%d", Cin, Cout, ks);
  return PAIG_E_UNSUPPORTED;
}

int paig_conv2d_wgrad_pf(const float* x, long long x_fs, int x_grp, long long x_gs, const float* dy, long long dy_fs,
                         const float* dpool, long long dpool_fs, const unsigned char* pcode, long long pcode_fs,
                         float* slab, int nblk_max, int* nblk_out, int F, int Cin, int Cout, int H, int W, int ks,
                         int flags, const float* xmax, int xmax_n, void* stream) {
  *nblk_out = 0;
  if (F <= 0) return 0;
  PAIG_REQUIRE((flags & 64) && (flags & 128) && dpool && pcode,
               "paig_conv2d_wgrad_pf: needs flags 64 | 128, the pooled gradient and the window codes");
  int rc = 0;
  if (paig_conv_split_wgrad(FView{x, x_fs, x_gs, x_grp}, FView{dy, dy_fs, 0, 0}, slab, nblk_max, nblk_out, F, Cin, Cout,
                            H, W, ks, flags, (hipStream_t)stream, &rc, XMax{const_cast<float*>(xmax), xmax_n},
                            PoolOut{const_cast<float*>(dpool), dpool_fs, const_cast<unsigned char*>(pcode), pcode_fs}))
    return rc;
  paig_set_error("paig_conv2d_wgrad_pf: no pool-fold instantiation for Cin=%d Cout=%d H=%d", Cin, Cout, H);
  return PAIG_E_UNSUPPORTED;
}

}  // extern "C"
