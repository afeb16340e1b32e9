// U-Net convolutions as implicit GEMMs on CDNA4 matrix cores
// (v_mfma_f32_16x16x4_f32: exact fp32 FMA chain, one instruction per 16
// FMAs per lane).  Reference: aten conv2d / convolution_backward behind
// nn/network/blocks.py:246-276 (ShallowUNet) and :113-170 (UNet).
//
// forward / dgrad   D[pixel][co] = im2col(X)[pixel][k] * Wt[k][co]
//   k = tap * CINP + ci (tap-major, 4 consecutive input channels per MFMA
//   k-step).  A fragment = one LDS read per lane at (lane pixel base +
//   compile-time (ci, tap) offset): zero VALU address math per MFMA; the
//   16 pixels of an M-tile are consecutive in (frame,row,x) order so each
//   lane's 4 accumulator rows are 4 adjacent x -> one float4 store.
//   Weights are staged once per block as Wt[tap][ci][co] (dgrad stages the
//   transposed + flipped kernel, so the same kernel computes dX).
// wgrad             D[co][n] = dY[co][pixel] * im2col(X)[pixel][n],
//   n = ci*KK + tap (the weight layout), K = pixels: each block walks many
//   (frame,rows) tiles accumulating in registers, waves split the pixels (and
//   the n-tiles when accumulators would not fit), one deterministic
//   cross-wave reduction, one partial row per block (paig_slab_reduce*).
// LDS layouts are padded so every fragment read is bank-conflict free
// (lanes 0-15 and 16-31 of a ds_read_b32 group land on disjoint halves).
#include "conv_tile.h"

namespace {

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ============================================================ forward / dgrad
template <int CIN, int COUT, int H, int W, int KS, bool DG>
struct FwdCfg {
  static constexpr int KK = KS * KS, PADL = KS / 2;
  static constexpr int CINP = ceil_div(CIN, 4) * 4;
  static constexpr int NT = ceil_div(COUT, 16);
  static constexpr int COUTP = pad16mod32(COUT);            // weight row stride, = 16 mod 32
  static constexpr int MW = W >= 32 ? 8 : (W >= 16 ? 4 : 2);  // M-tiles per wave
  static constexpr int TPX = 4 * MW * 16;                    // pixels per block tile
  static constexpr int FPT = TPX >= H * W ? TPX / (H * W) : 1;
  static constexpr int RT = TPX >= H * W ? H : TPX / W;      // rows per tile (per frame)
  static constexpr int TWP = W + 8;                          // cols: [3]=halo, [4, 4+W)=data, [4+W]=halo
  static constexpr int ROWS = RT + KS - 1;
  static constexpr int CHS = to_mod32(ROWS * TWP, 16);        // channel stride in LDS, = 16 mod 32
  static constexpr int CI0 = CINP < 8 ? CINP : 8;
  static constexpr int CI = (FPT * CI0 * CHS * 4 > 48 * 1024 && CI0 > 4) ? 4 : CI0;
  static constexpr int NCH = CINP / CI;
  static constexpr int LDS_I = FPT * CI * CHS;
  static constexpr int LDS_W = KK * CINP * COUTP;
  static constexpr int LDS = (LDS_I + LDS_W) * 4;
  static_assert(CINP % CI == 0, "chunking");
  static_assert(W % 4 == 0 && (H * W) % 16 == 0, "MFMA conv needs W % 4 == 0");
  static_assert(RT * W * FPT == TPX || RT == H, "tile");
};

template <int CIN, int COUT, int H, int W, int KS, bool DG, bool UPS>
__global__ void __launch_bounds__(256)
conv_fwd_mfma_k(FView in, FViewW out, FView aux, const float* __restrict__ w, const float* __restrict__ bias, int F,
                int flags, int ntiles) {
  constexpr long long PLANE = UPS ? (long long)(H / 2) * (W / 2) : (long long)H * W;
  using C = FwdCfg<CIN, COUT, H, W, KS, DG>;
  constexpr int KK = C::KK, NT = C::NT, MW = C::MW, TWP = C::TWP, CHS = C::CHS, CI = C::CI;
  constexpr int RT = C::RT, FPT = C::FPT, ROWS = C::ROWS, COUTP = C::COUTP, CINP = C::CINP, NCH = C::NCH;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* Il = lds;                 // [FPT][CI][CHS]
  float* Wl = lds + C::LDS_I;      // [KK][CINP][COUTP]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  constexpr int NRB = H / RT;      // row blocks per frame (RT divides H)
  constexpr int Q = W / 4;         // float4 per row
  constexpr int NI = FPT * CI * ROWS * Q;   // staged 4-pixel segments per (tile, chunk)
  constexpr int NL = (NI + 255) / 256;

  // ---- weights -> Wt[tap][ci][co] (zero padded); dgrad: transposed + flipped.
  // Staged once: the block is persistent over tiles.
  for (int i = tid; i < KK * CINP * COUTP; i += 256) {
    const int co = i % COUTP;
    const int ci = (i / COUTP) % CINP;
    const int tap = i / (COUTP * CINP);
    float v = 0.f;
    if (co < COUT && ci < CIN) {
      if (DG) v = w[(ci * COUT + co) * KK + (KK - 1 - tap)];
      else v = w[(co * CIN + ci) * KK + tap];
    }
    Wl[i] = v;
  }
  // ---- zero the halo columns (never written by the staging below)
  for (int i = tid; i < FPT * CI * ROWS; i += 256) {
    Il[(i / ROWS) * CHS + (i % ROWS) * TWP + 3] = 0.f;
    Il[(i / ROWS) * CHS + (i % ROWS) * TWP + 4 + W] = 0.f;
  }

  // ---- per-lane pixel bases of this wave's M-tiles
  int abase[MW];
#pragma unroll
  for (int mt = 0; mt < MW; ++mt) {
    const int pix = (wv * MW + mt) * 16 + (lane & 15);     // pixel index within the tile
    const int fi = pix / (RT * W);
    const int rem = pix % (RT * W);
    const int y = rem / W, x = rem % W;
    abase[mt] = fi * CI * CHS + (lane >> 4) * CHS + y * TWP + x + 4 - C::PADL;
  }

  // ---- software pipeline: the global loads of (tile, chunk + 1) -- or of the
  // block's next tile -- are in flight while the current chunk is multiplied
  Seg<UPS, H, W> seg[NL];
  auto issue = [&](int t, int ch) {
    const int tt = (UPS && H >= 32) ? opaque(tid) : tid;
    const int f0 = (t / NRB) * FPT, y0 = (t % NRB) * RT;
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int i = tt + l * 256;
      const int q = i % Q, r = i / Q;
      const int rr = r % ROWS, c = (r / ROWS) % CI, fi = r / (ROWS * CI);
      const int f = f0 + fi, gy = y0 + rr - C::PADL, ci = ch * CI + c;
      const bool ok = i < NI && f < F && gy >= 0 && gy < H && ci < CIN;
      seg[l].issue(ok ? in.frame(f) + ci * PLANE : in.p, gy, q, ok);
    }
  };
  auto commit = [&](int t) {
    const int tt = (UPS && H >= 32) ? opaque(tid) : tid;
    const int y0 = (t % NRB) * RT;
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int i = tt + l * 256;
      if (NI % 256 != 0 && i >= NI) break;
      const int q = i % Q, r = i / Q;
      const int rr = r % ROWS, c = (r / ROWS) % CI, fi = r / (ROWS * CI);
      *reinterpret_cast<f32x4*>(&Il[(fi * CI + c) * CHS + rr * TWP + 4 + 4 * q]) =
          seg[l].finish(y0 + rr - C::PADL, q);
    }
  };

  constexpr long long HW = (long long)H * W;
  // the full-resolution upsampling convs hold 8 raw floats per segment: their
  // prefetch would cost the occupancy it is meant to replace (measured), so
  // they load synchronously
  constexpr bool PIPE = !(UPS && H >= 32);
  int tile = blockIdx.x;
  if (PIPE && tile < ntiles) issue(tile, 0);
  for (; tile < ntiles; tile += gridDim.x) {
    const int f0 = (tile / NRB) * FPT;
    const int y0 = (tile % NRB) * RT;
    f32x4 acc[MW][NT];
#pragma unroll
    for (int mt = 0; mt < MW; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int ch = 0; ch < NCH; ++ch) {
      const int ci0 = ch * CI;
      __syncthreads();           // previous chunk's fragment reads are done
      if (!PIPE) issue(tile, ch);
      commit(tile);
      __syncthreads();
      if (PIPE) {
        if (ch + 1 < NCH) issue(tile, ch + 1);
        else if (tile + (int)gridDim.x < ntiles) issue(tile + gridDim.x, 0);
      }
#pragma unroll
      for (int tap = 0; tap < KK; ++tap) {
        const int toff = (tap / KS) * TWP + (tap % KS);
#pragma unroll
        for (int cg = 0; cg < CI / 4; ++cg) {
          float b[NT];
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
            b[nt] = Wl[(tap * CINP + ci0 + cg * 4 + (lane >> 4)) * COUTP + nt * 16 + (lane & 15)];
#pragma unroll
          for (int mt = 0; mt < MW; ++mt) {
            const float a = Il[abase[mt] + cg * 4 * CHS + toff];
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma4(a, b[nt], acc[mt][nt]);
          }
        }
      }
    }

    // ---- epilogue: lane holds pixels (lane>>4)*4 + r of each M-tile for co = nt*16 + (lane&15)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int co = nt * 16 + (lane & 15);
      if (co >= COUT) continue;
      const float bv = bias ? bias[co] : 0.f;
#pragma unroll
      for (int mt = 0; mt < MW; ++mt) {
        const int pix = (wv * MW + mt) * 16 + (lane >> 4) * 4;
        const int fi = pix / (RT * W);
        const int rem = pix % (RT * W);
        const int y = y0 + rem / W, x = rem % W;
        const int f = f0 + fi;
        if (f >= F || y >= H) continue;
        float* op = out.frame(f) + co * HW + (long long)y * W + x;
        f32x4 v = acc[mt][nt];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += bv;
        if (flags & 1) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = v[r] < 0.f ? 0.f : v[r];
        }
        if (flags & 4) {
          const f32x4 o = *reinterpret_cast<const f32x4*>(op);
          v += o;
        }
        if (flags & 2) {
          const f32x4 m = *reinterpret_cast<const f32x4*>(aux.frame(f) + co * HW + (long long)y * W + x);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = m[r] > 0.f ? v[r] : 0.f;
        }
        *reinterpret_cast<f32x4*>(op) = v;
      }
    }
  }
}

// ===================================================================== wgrad
template <int CIN, int COUT, int H, int W, int KS>
struct WgCfg {
  static constexpr int KK = KS * KS, PADL = KS / 2;
  static constexpr int NCOL = CIN * KK;
  static constexpr int NT = ceil_div(NCOL, 16);
  static constexpr int MT = ceil_div(COUT, 16);
  static constexpr int WN = (MT * NT * 4 <= 96) ? 1 : ((MT * ceil_div(NT, 2) * 4 <= 96) ? 2 : 4);
  static constexpr int WP = 4 / WN;
  static constexpr int NTW = ceil_div(NT, WN);
  static constexpr int TWP = W + 8;
  // rows per tile: as many as fit ~48 KB of LDS
  static constexpr int COP = pad16mod32(COUT);
  static constexpr int rows_fit(int rt) {
    return (CIN * to_mod32((rt + KS - 1) * TWP, 2) + rt * W * COP) * 4 <= 56 * 1024 ? rt : rows_fit(rt / 2);
  }
  static constexpr int RT0 = rows_fit(H);
  static constexpr int FPT = (RT0 == H && H * W < 256) ? 256 / (H * W) : 1;
  static constexpr int RT = RT0;
  static constexpr int ROWS = RT + KS - 1;
  static constexpr int CHS = to_mod32(ROWS * TWP, 2);
  static constexpr int LDS_X = FPT * CIN * CHS;
  static constexpr int LDS_D = FPT * RT * W * COP;
  static constexpr int RED = 4 * 64 * MT * NTW * 4;          // cross-wave reduction buffer
  static constexpr int LDS = ((LDS_X + LDS_D) > RED ? (LDS_X + LDS_D) : RED) * 4;
  static constexpr int NG = FPT * RT * W / 4;                // 4-pixel groups per tile
  static constexpr int SLAB = COUT * NCOL + COUT;
  static_assert(W % 4 == 0, "W % 4");
  static_assert(H % RT == 0, "RT divides H");
};

template <int CIN, int COUT, int H, int W, int KS, bool UPS>
__global__ void __launch_bounds__(256)
conv_wgrad_mfma_k(FView x, FView dy, float* __restrict__ slab, int F, int ntiles) {
  using C = WgCfg<CIN, COUT, H, W, KS>;
  // staging index math recomputed (opaque) rather than hoisted where that
  // buys a wave of occupancy -- measured per shape (r01 profiles)
  constexpr bool WG_OPQ = (H == 16 && (CIN == 16 || UPS)) || (UPS && H >= 32);
  constexpr long long PLANE = UPS ? (long long)(H / 2) * (W / 2) : (long long)H * W;
  constexpr int KK = C::KK, NT = C::NT, MT = C::MT, WN = C::WN, WP = C::WP, NTW = C::NTW;
  constexpr int TWP = C::TWP, CHS = C::CHS, RT = C::RT, FPT = C::FPT, ROWS = C::ROWS, COP = C::COP;
  constexpr int NCOL = C::NCOL;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* Xl = lds;                 // [FPT][CIN][CHS]
  float* Dl = lds + C::LDS_X;      // [FPT*RT*W][COP]  (pixel-major, co fastest)
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wn = wv % WN, wp = wv / WN;

  // per-lane column offsets (n = ci*KK + tap) of this wave's n-tiles
  int coff[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    int n = (wn + j * WN) * 16 + (lane & 15);
    if (n >= NCOL) n = NCOL - 1;                  // padded columns read valid LDS, never stored
    const int ci = n / KK, tap = n % KK;
    coff[j] = ci * CHS + (tap / KS) * TWP + (tap % KS) + 4 - C::PADL;
  }
  f32x4 acc[MT][NTW];
  float bacc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    bacc[m] = 0.f;
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[m][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // zero halo columns once
  for (int i = tid; i < FPT * CIN * ROWS; i += 256) {
    Xl[(i / ROWS) * CHS + (i % ROWS) * TWP + 3] = 0.f;
    Xl[(i / ROWS) * CHS + (i % ROWS) * TWP + 4 + W] = 0.f;
  }
  if (COP > COUT) {   // zero padded co columns once (read by padded M rows; never stored)
    for (int i = tid; i < FPT * RT * W * (COP - COUT); i += 256)
      Dl[(i / (COP - COUT)) * COP + COUT + i % (COP - COUT)] = 0.f;
  }
  constexpr int NRB = H / RT;
  constexpr int Q = W / 4;
  constexpr int NIX = FPT * CIN * ROWS * Q, NLX = (NIX + 255) / 256;   // X row segments per tile
  constexpr int NID = FPT * COUT * RT * Q, NLD = (NID + 255) / 256;    // dY segments per tile
  // software pipeline: the next tile's global loads are in flight while the
  // current tile is multiplied
  Seg<UPS, H, W> sx[NLX];
  f32x4 sd[NLD];
  auto issue = [&](int t) {
    const int tt = WG_OPQ ? opaque(tid) : tid;
    const int f0 = (t / NRB) * FPT, y0 = (t % NRB) * RT;
#pragma unroll
    for (int l = 0; l < NLX; ++l) {
      const int i = tt + l * 256;
      const int q = i % Q, r = i / Q;
      const int rr = r % ROWS, c = (r / ROWS) % CIN, fi = r / (ROWS * CIN);
      const int f = f0 + fi, gy = y0 + rr - C::PADL;
      const bool ok = i < NIX && f < F && gy >= 0 && gy < H;
      sx[l].issue(ok ? x.frame(f) + c * PLANE : x.p, gy, q, ok);
    }
#pragma unroll
    for (int l = 0; l < NLD; ++l) {
      const int i = tt + l * 256;
      const int co = i % COUT, r = i / COUT;
      const int q = r % Q, rr = (r / Q) % RT, fi = r / (Q * RT);
      const int f = f0 + fi;
      sd[l] = (i < NID && f < F)
                  ? *reinterpret_cast<const f32x4*>(dy.frame(f) + ((long long)co * H + y0 + rr) * W + 4 * q)
                  : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto commit = [&](int t) {
    const int tt = WG_OPQ ? opaque(tid) : tid;
    const int y0 = (t % NRB) * RT;
#pragma unroll
    for (int l = 0; l < NLX; ++l) {
      const int i = tt + l * 256;
      if (NIX % 256 != 0 && i >= NIX) break;
      const int q = i % Q, r = i / Q;
      const int rr = r % ROWS, c = (r / ROWS) % CIN, fi = r / (ROWS * CIN);
      *reinterpret_cast<f32x4*>(&Xl[(fi * CIN + c) * CHS + rr * TWP + 4 + 4 * q]) =
          sx[l].finish(y0 + rr - C::PADL, q);
    }
    // dY -> [pixel][co]: co varies fastest across lanes so the transposed LDS
    // writes of one float4 (4 pixels) are conflict free
#pragma unroll
    for (int l = 0; l < NLD; ++l) {
      const int i = tt + l * 256;
      if (NID % 256 != 0 && i >= NID) break;
      const int co = i % COUT, r = i / COUT;
      const int q = r % Q, rr = (r / Q) % RT, fi = r / (Q * RT);
      const int pb = (fi * RT + rr) * W + 4 * q;
#pragma unroll
      for (int e = 0; e < 4; ++e) Dl[(pb + e) * COP + co] = sd[l][e];
    }
  };
  constexpr bool PIPE = true;
  if (PIPE && (int)blockIdx.x < ntiles) issue(blockIdx.x);
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    __syncthreads();            // previous tile's fragment reads are done
    if (!PIPE) issue(tile);
    commit(tile);
    __syncthreads();
    if (PIPE && tile + (int)gridDim.x < ntiles) issue(tile + gridDim.x);
    // a wave takes whole rows (FPT*RT rows per tile, split over the WP pixel
    // waves); the Q 4-pixel groups of a row are unrolled so the fragment
    // reads of later groups are in flight behind the MFMAs of earlier ones
    // (waves holding 18+ accumulator tiles keep the row loop rolled: the
    // unrolled form's in-flight fragments would cost them occupancy)
    constexpr int UNQ = Q;
#pragma unroll 1
    for (int rr = wp; rr < FPT * RT; rr += WP) {
      const int pixrow = rr * W + (lane >> 4);   // (fi*RT + y)*W
      const int xrow = (rr / RT) * CIN * CHS + (rr % RT) * TWP + (lane >> 4);
#pragma unroll UNQ
      for (int q = 0; q < Q; ++q) {
        const int pix = pixrow + 4 * q;
        float a[MT];
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          a[m] = Dl[pix * COP + m * 16 + (lane & 15)];
          bacc[m] += a[m];
        }
        const int xb = xrow + 4 * q;
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
          if (wn + j * WN < NT) {
            const float b = Xl[coff[j] + xb];
#pragma unroll
            for (int m = 0; m < MT; ++m) acc[m][j] = mfma4(a[m], b, acc[m][j]);
          }
        }
      }
    }
  }
  __syncthreads();
  // ---- cross-wave reduction (waves with equal wn, different wp) through LDS
  float* R = lds;   // [4 waves][MT][NTW][4][64]
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) R[(((wv * MT + m) * NTW + j) * 4 + r) * 64 + lane] = acc[m][j][r];
  // bias: lane (l&15) co partial over its (l>>4) pixel lanes, then across waves
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    float v = bacc[m];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    bacc[m] = v;
  }
  __syncthreads();
  float* s = slab + (long long)blockIdx.x * C::SLAB;
  if (wp == 0) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        const int nt = wn + j * WN;
        if (nt >= NT) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = 0.f;
          for (int p = 0; p < WP; ++p) v += R[((((p * WN + wn) * MT + m) * NTW + j) * 4 + r) * 64 + lane];
          const int co = m * 16 + (lane >> 4) * 4 + r;
          const int n = nt * 16 + (lane & 15);
          if (co < COUT && n < NCOL) s[co * NCOL + n] = v;
        }
      }
  }
  __syncthreads();
  // bias partials: every wave with wn == 0 holds a full-pixel-subset partial
  if (wn == 0 && lane < 16) {
#pragma unroll
    for (int m = 0; m < MT; ++m) R[(wp * MT + m) * 16 + lane] = bacc[m];
  }
  __syncthreads();
  if (tid < COUT) {
    const int m = tid / 16, l = tid % 16;
    float v = 0.f;
    for (int p = 0; p < WP; ++p) v += R[(p * MT + m) * 16 + l];
    s[COUT * NCOL + tid] = v;
  }
}

template <int CIN, int COUT, int H, int W, int KS, bool DG, bool UPS>
static int fwd_launch(FView in, FViewW out, FView aux, const float* w, const float* b, int F, int flags,
                      hipStream_t st) {
  using C = FwdCfg<CIN, COUT, H, W, KS, DG>;
  constexpr int NRB = H / C::RT;
  const int ntiles = cdiv(F, C::FPT) * NRB;
  auto k = conv_fwd_mfma_k<CIN, COUT, H, W, KS, DG, UPS>;
  static int resident = 0;
  if (!resident) {
    if (C::LDS > 64 * 1024)
      (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    resident = persistent_grid((const void*)k, C::LDS);
  }
  const int nb = ntiles < resident ? ntiles : resident;
  hipLaunchKernelGGL(k, dim3(nb), dim3(256), C::LDS, st, in, out, aux, w, b, F, flags, ntiles);
  PAIG_CHECK_LAUNCH();
  return 0;
}

// ====================================== forward / dgrad, Cout = 8: pixel pairs
// A 16x16 MFMA tile with only 8 output channels idles half its columns.  Here
// a D row is a PAIR of horizontally adjacent output pixels (x = 2p, 2p+1) and
// the 16 columns are (s, co), s = which pixel of the pair:
//   D[p][(s,co)] = sum_{ci,dy,dx'} X[ci][y+dy-1][2p+dx'] * B[(ci,dy,dx')][(s,co)],
//   dx' in {-1,0,1,2},  B = w[co][ci][dy][dx'-s]  (0 where dx'-s is outside -1..1)
// K per input channel is 3 rows x 4 columns (12 instead of 9) for twice the
// output per MFMA: 2/3 of the MFMAs of the plain layout.  One MFMA k-step is
// (ci, dy); its 4 k-values are the 4 dx', i.e. lane group g = lane>>4 reads
// x = 2p + g - 1: lanes 0-31 and 32-63 each read 32 CONSECUTIVE floats of one
// LDS row (conflict-free for any pitch).  The weights of all k-steps live in
// VGPRs for the whole (persistent) block.  Epilogue: lanes (s=0,co) and
// (s=1,co) trade values (xor 8) so each stores one float4 of 4 adjacent pixels.
template <int CIN, int H, int W, bool DG>
struct PairCfg {
  static constexpr int COUT = 8, KS = 3, PADL = 1, KK = 9;
  static constexpr int PPR = W / 2;                       // pairs per row
  static_assert(W % 8 == 0 && (PPR % 16 == 0 || 16 % PPR == 0), "pair tiling");
  static constexpr int RPM = 16 / PPR > 0 ? 16 / PPR : 1; // rows per M-tile (16 pairs)
  static constexpr int MTR = PPR / 16 > 0 ? PPR / 16 : 1; // M-tiles per row
  static constexpr int MW = 4;                            // M-tiles per wave
  static constexpr int TPAIRS = 4 * MW * 16;              // pairs per block tile
  static constexpr int TPX = 2 * TPAIRS;
  static constexpr int FPT = TPX >= H * W ? TPX / (H * W) : 1;
  static constexpr int RT = TPX >= H * W ? H : TPX / W;
  static constexpr int ROWS = RT + 2;
  // row pitch: >= W + 5 (x from -1 to W), 16B-aligned rows; rows of one M-tile
  // (W < 32) land on disjoint bank ranges: pitch = 16 (mod 32) for 2 rows,
  // 8 (mod 32) for 4 rows
  static constexpr int TWP = RPM == 1 ? W + 8 : (RPM == 2 ? to_mod32(W + 8, 16) : to_mod32(W + 8, 8));
  static constexpr int CHS = ROWS * TWP;
  static constexpr int CI = CIN < 8 ? CIN : 8;            // channels per staged chunk
  static constexpr int NCH = (CIN + CI - 1) / CI;
  static constexpr int LDS = FPT * CI * CHS * 4;
  static_assert(RT * W * FPT == TPX || RT == H, "tile");
  static_assert(H % RT == 0, "RT divides H");
};

template <int CIN, int H, int W, bool DG>
__global__ void __launch_bounds__(256)
conv_fwd_pair_k(FView in, FViewW out, FView aux, const float* __restrict__ w, const float* __restrict__ bias, int F,
                int flags, int ntiles) {
  using C = PairCfg<CIN, H, W, DG>;
  constexpr int COUT = 8, MW = C::MW, TWP = C::TWP, CHS = C::CHS, CI = C::CI, NCH = C::NCH;
  constexpr int RT = C::RT, FPT = C::FPT, ROWS = C::ROWS, PPR = C::PPR, RPM = C::RPM, MTR = C::MTR;
  constexpr long long HW = (long long)H * W, PLANE = HW;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* Il = lds;   // [FPT][CI][ROWS][TWP], data at column 4 + x
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int g = lane >> 4;   // dx' = g - 1
  const int col = lane & 15, s = col >> 3, co = col & 7;
  constexpr int NRB = H / RT;
  constexpr int Q = W / 4;

  // ---- B fragments of every k-step (ci, dy) in registers
  float breg[CIN * 3];
#pragma unroll
  for (int ci = 0; ci < CIN; ++ci)
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const int dx = g - 1 - s;   // tap column in -1..1, else no contribution
      float v = 0.f;
      if (dx >= -1 && dx <= 1) {
        const int tap = dy * 3 + dx + 1;
        v = DG ? w[(ci * COUT + co) * 9 + (8 - tap)] : w[(co * CIN + ci) * 9 + tap];
      }
      breg[ci * 3 + dy] = v;
    }
  // ---- zero the halo columns (x = -1 and x = W .. W+3 are never staged)
  for (int i = tid; i < FPT * CI * ROWS; i += 256) {
    float* r = Il + (i / ROWS) * CHS + (i % ROWS) * TWP;
    r[3] = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) r[4 + W + e] = 0.f;
  }
  // ---- per-lane A base (pair p of M-tile mt -> row, x = 2*(p % PPR) + dx')
  int abase[MW];
#pragma unroll
  for (int mt = 0; mt < MW; ++mt) {
    const int tile_m = wv * MW + mt;                 // M-tile index within the block tile
    const int p = (tile_m % MTR) * 16 + col;         // pair within its row group
    const int rowg = (tile_m / MTR) * RPM + p / PPR; // row within the block tile (all frames)
    const int fi = rowg / RT, y = rowg % RT;
    abase[mt] = fi * CI * CHS + y * TWP + 2 * (p % PPR) + g + 3;   // 4 + x + dx', dx' = g - 1
  }

  constexpr int NI = FPT * CI * ROWS * Q, NL = (NI + 255) / 256;
  Seg<false, H, W> seg[NL];
  auto issue = [&](int t, int ch) {
    const int f0 = (t / NRB) * FPT, y0 = (t % NRB) * RT;
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int i = tid + l * 256;
      const int q = i % Q, r = i / Q;
      const int rr = r % ROWS, c = (r / ROWS) % CI, fi = r / (ROWS * CI);
      const int f = f0 + fi, gy = y0 + rr - 1, ci = ch * CI + c;
      const bool ok = i < NI && f < F && gy >= 0 && gy < H && ci < CIN;
      seg[l].issue(ok ? in.frame(f) + ci * PLANE : in.p, gy, q, ok);
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int i = tid + l * 256;
      if (NI % 256 != 0 && i >= NI) break;
      const int q = i % Q, r = i / Q;
      const int rr = r % ROWS, c = (r / ROWS) % CI, fi = r / (ROWS * CI);
      *reinterpret_cast<f32x4*>(&Il[(fi * CI + c) * CHS + rr * TWP + 4 + 4 * q]) = seg[l].finish(0, q);
    }
  };

  int tile = blockIdx.x;
  if (tile < ntiles) issue(tile, 0);
  for (; tile < ntiles; tile += gridDim.x) {
    const int f0 = (tile / NRB) * FPT, y0 = (tile % NRB) * RT;
    f32x4 acc[MW];
#pragma unroll
    for (int mt = 0; mt < MW; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      __syncthreads();
      commit();
      __syncthreads();
      if (ch + 1 < NCH) issue(tile, ch + 1);
      else if (tile + (int)gridDim.x < ntiles) issue(tile + gridDim.x, 0);
#pragma unroll
      for (int c = 0; c < CI; ++c) {
        if (ch * CI + c >= CIN) break;
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) {
          const float b = breg[(ch * CI + c) * 3 + dy];
#pragma unroll
          for (int mt = 0; mt < MW; ++mt)
            acc[mt] = mfma4(Il[abase[mt] + c * CHS + dy * TWP], b, acc[mt]);
        }
      }
    }
    // ---- epilogue: lane holds pairs p = (lane>>4)*4 + r of each M-tile for (s, co)
    const float bv = bias ? bias[co] : 0.f;
#pragma unroll
    for (int mt = 0; mt < MW; ++mt) {
      float o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float mine = acc[mt][r];
        const float other = __shfl_xor(mine, 8, 64);
        o[r] = mine;
        acc[mt][r] = other;   // partner's value for the same pair
      }
      // s = 0: pixels 2p0 .. 2p0+3 ; s = 1: pixels 2p0+4 .. 2p0+7
      f32x4 v;
      if (s == 0) v = f32x4{o[0], acc[mt][0], o[1], acc[mt][1]};
      else v = f32x4{acc[mt][2], o[2], acc[mt][3], o[3]};
      const int tile_m = wv * MW + mt;
      const int p0 = (tile_m % MTR) * 16 + (lane >> 4) * 4;
      const int rowg = (tile_m / MTR) * RPM + p0 / PPR;
      const int fi = rowg / RT, y = y0 + rowg % RT, x = 2 * (p0 % PPR) + 4 * s;
      const int f = f0 + fi;
      if (f >= F) continue;
      float* op = out.frame(f) + co * HW + (long long)y * W + x;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] += bv;
      if (flags & 1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = v[e] < 0.f ? 0.f : v[e];
      }
      if (flags & 4) v += *reinterpret_cast<const f32x4*>(op);
      if (flags & 2) {
        const f32x4 m = *reinterpret_cast<const f32x4*>(aux.frame(f) + co * HW + (long long)y * W + x);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = m[e] > 0.f ? v[e] : 0.f;
      }
      *reinterpret_cast<f32x4*>(op) = v;
    }
  }
}

template <int CIN, int H, int W, bool DG>
static int pair_launch(FView in, FViewW out, FView aux, const float* w, const float* b, int F, int flags,
                       hipStream_t st) {
  using C = PairCfg<CIN, H, W, DG>;
  const int ntiles = cdiv(F, C::FPT) * (H / C::RT);
  auto k = conv_fwd_pair_k<CIN, H, W, DG>;
  static int resident = 0;
  if (!resident) {
    if (C::LDS > 64 * 1024)
      (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    resident = persistent_grid((const void*)k, C::LDS);
  }
  const int nb = ntiles < resident ? ntiles : resident;
  hipLaunchKernelGGL(k, dim3(nb), dim3(256), C::LDS, st, in, out, aux, w, b, F, flags, ntiles);
  PAIG_CHECK_LAUNCH();
  return 0;
}

template <int CIN, int COUT, int H, int W, int KS, bool UPS>
static int wgrad_launch(FView x, FView dy, float* slab, int nblk_max, int* nblk_out, int F, hipStream_t st) {
  using C = WgCfg<CIN, COUT, H, W, KS>;
  const int ntiles = cdiv(F, C::FPT) * (H / C::RT);
  auto k = conv_wgrad_mfma_k<CIN, COUT, H, W, KS, UPS>;
  static int resident = 0;
  if (!resident) {
    if (C::LDS > 64 * 1024)
      (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    resident = persistent_grid((const void*)k, C::LDS);
  }
  int nb = ntiles < nblk_max ? ntiles : nblk_max;   // one wave of co-resident blocks
  if (nb > resident) nb = resident;
  if (nb < 1) nb = 1;
  *nblk_out = nb;
  hipLaunchKernelGGL(k, dim3(nb), dim3(256), C::LDS, st, x, dy, slab, F, ntiles);
  PAIG_CHECK_LAUNCH();
  return 0;
}

// (CIN, COUT, H, KS): ShallowUNet(hidden 8) at 32x32 -- forward and dgrad
// shapes (dgrad kernel shapes are (layer Cout, layer Cin)); *_UP: convs whose
// input is the fused 2x upsample (c7, c10).
#define PAIG_MFMA_FWD(X)                                                                                  \
  X(3, 8, 32, 3) X(8, 8, 32, 3) X(8, 16, 16, 3) X(16, 16, 16, 3) X(16, 32, 8, 3) X(32, 32, 8, 3)         \
  X(32, 16, 16, 3) X(16, 16, 32, 3) X(24, 8, 32, 3) X(8, 2, 32, 1) X(16, 8, 16, 3) X(8, 24, 32, 3)       \
  X(2, 8, 32, 1) X(32, 16, 8, 3) X(16, 32, 16, 3)
#define PAIG_MFMA_WG(X)                                                                                   \
  X(3, 8, 32, 3) X(8, 8, 32, 3) X(8, 16, 16, 3) X(16, 16, 16, 3) X(16, 32, 8, 3) X(32, 32, 8, 3)         \
  X(32, 16, 16, 3) X(16, 16, 32, 3) X(24, 8, 32, 3) X(8, 2, 32, 1)
#define PAIG_MFMA_UP(X) X(32, 16, 16, 3) X(16, 16, 32, 3)
// (CIN, H) of the Cout = 8, 3x3 shapes on the pixel-pair kernel (fwd: c1, c2,
// c11, c12; dgrad: c2/c12 (8 -> 8 at 32) and c3 (16 -> 8 at 16))
#define PAIG_MFMA_PAIR(X) X(3, 32) X(8, 32) X(24, 32) X(16, 16)

}  // namespace

// Returns 1 if handled (rc in *rc), 0 if the shape has no MFMA instantiation.
// flags: 1 relu, 2 mask(aux>0), 4 accumulate, 8 dgrad, 32 input = 2x upsample of (H/2 x W/2)
int paig_conv_mfma_fwd(FView in, FViewW out, FView aux, const float* w, const float* b, int F, int Cin, int Cout,
                       int H, int W, int ks, int flags, hipStream_t st, int* rc, XMax xm, const void* wp,
                       PoolOut pout) {
  if ((flags & (128 | 256)) &&
      paig_conv_split_fwd(in, out, aux, w, b, F, Cin, Cout, H, W, ks, flags, st, rc, xm, wp, pout))
    return 1;
  if (flags & 64) {
    paig_set_error("paig_conv2d_fwd: the fused pool (flags & 64) needs a split-path shape");
    *rc = PAIG_E_UNSUPPORTED;
    return 1;
  }
  const bool dg = (flags & 8) != 0;
  const bool up = (flags & 32) != 0;
  const int fl = flags & 7;
  if (H != W) return 0;
  if (up) {
    if (dg) return 0;
#define PAIG_CASE(CI, CO, HH, K)                                                              \
    if (Cin == CI && Cout == CO && H == HH && ks == K) {                                      \
      *rc = fwd_launch<CI, CO, HH, HH, K, false, true>(in, out, aux, w, b, F, fl, st);        \
      return 1;                                                                               \
    }
    PAIG_MFMA_UP(PAIG_CASE)
#undef PAIG_CASE
    return 0;
  }
  if (Cout == 8 && ks == 3 && !(flags & 64)) {
#define PAIG_PCASE(CI, HH)                                                                   \
    if (Cin == CI && H == HH) {                                                              \
      *rc = dg ? pair_launch<CI, HH, HH, true>(in, out, aux, w, b, F, fl, st)                \
               : pair_launch<CI, HH, HH, false>(in, out, aux, w, b, F, fl, st);              \
      return 1;                                                                              \
    }
    PAIG_MFMA_PAIR(PAIG_PCASE)
#undef PAIG_PCASE
  }
#define PAIG_CASE(CI, CO, HH, K)                                                                      \
  if (Cin == CI && Cout == CO && H == HH && ks == K) {                                                \
    *rc = dg ? fwd_launch<CI, CO, HH, HH, K, true, false>(in, out, aux, w, b, F, fl, st)              \
             : fwd_launch<CI, CO, HH, HH, K, false, false>(in, out, aux, w, b, F, fl, st);            \
    return 1;                                                                                         \
  }
  PAIG_MFMA_FWD(PAIG_CASE)
#undef PAIG_CASE
  return 0;
}

int paig_conv_mfma_wgrad(FView x, FView dy, float* slab, int nblk_max, int* nblk_out, int F, int Cin, int Cout, int H,
                         int W, int ks, int flags, hipStream_t st, int* rc, XMax xm) {
  if ((flags & (128 | 256)) &&
      paig_conv_split_wgrad(x, dy, slab, nblk_max, nblk_out, F, Cin, Cout, H, W, ks, flags, st, rc, xm))
    return 1;
  if (H != W) return 0;
  if (flags & 32) {
#define PAIG_CASE(CI, CO, HH, K)                                                                 \
    if (Cin == CI && Cout == CO && H == HH && ks == K) {                                         \
      *rc = wgrad_launch<CI, CO, HH, HH, K, true>(x, dy, slab, nblk_max, nblk_out, F, st);       \
      return 1;                                                                                  \
    }
    PAIG_MFMA_UP(PAIG_CASE)
#undef PAIG_CASE
    return 0;
  }
#define PAIG_CASE(CI, CO, HH, K)                                                         \
  if (Cin == CI && Cout == CO && H == HH && ks == K) {                                   \
    *rc = wgrad_launch<CI, CO, HH, HH, K, false>(x, dy, slab, nblk_max, nblk_out, F, st); \
    return 1;                                                                            \
  }
  PAIG_MFMA_WG(PAIG_CASE)
#undef PAIG_CASE
  return 0;
}

// Query (see include/paig_hip.h): does paig_conv2d_fwd (what = 0) or
// paig_conv2d_wgrad (what = 1) run this shape on the MFMA path with these
// flags?  flags & 32 (fused 2x upsample input) exists ONLY on that path, so
// the host uses this to decide which upsamples it may fuse.
extern "C" int paig_conv2d_mfma_supported(int what, int Cin, int Cout, int H, int W, int ks, int flags) {
  if ((flags & (128 | 256)) && paig_conv_split_supported(what, Cin, Cout, H, W, ks, flags)) return 1;
  if (flags & 64) return 0;   // the fused pool exists on the split path only
  if (H != W) return 0;
  const bool up = (flags & 32) != 0, dg = (flags & 8) != 0;
#define PAIG_CASE(CI, CO, HH, K) \
  if (Cin == CI && Cout == CO && H == HH && ks == K) return 1;
  if (up) {
    if (dg) return 0;
    PAIG_MFMA_UP(PAIG_CASE)
    return 0;
  }
  if (what == 0) {
    PAIG_MFMA_FWD(PAIG_CASE)
  } else {
    PAIG_MFMA_WG(PAIG_CASE)
  }
#undef PAIG_CASE
  return 0;
}
