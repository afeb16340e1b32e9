// U-Net convolutions on the gfx950 16-bit matrix cores with split-precision
// operands (v_mfma_f32_16x16x32_{f16,bf16}, fp32 accumulate).  Reference:
// aten conv2d / convolution_backward behind nn/network/blocks.py:246-276
// (ShallowUNet) and :113-170 (UNet).
//
// Every fp32 operand v is split as v = hi + lo with hi = rn16(v) and
// lo = rn16(v - hi) (the subtraction is exact in fp32), and a product is
// formed from three MFMAs: hi*hi + hi*lo + lo*hi (the lo*lo term and the
// residual of lo are below fp32 accumulation noise for f16 pieces).  Per K
// element a 16x16x32 MFMA costs 1/16 of the f32-input v_mfma_f32_16x16x4_f32,
// so the three-term product does fp32-accurate convolutions at ~5x the f32
// matrix rate; these layers (3..128 channels) then run at the HBM/LDS
// roofline instead of the MFMA one.  Precision modes (PM):
//   0  f16 hi/lo   (22 significant bits).  Every operand is scaled by a
//                  power of two into f16's top binade: forward activations
//                  and dgrad gradients per tile (the tile's outputs are
//                  complete, the epilogue scales back), weights per output
//                  channel (paig_conv_wprep's header, or the block's own
//                  staging), wgrad X by the forward's recorded maximum and
//                  dY by a running block exponent (whose pixel sums span
//                  tiles: a tile needing a smaller exponent first rescales
//                  the accumulators, exactly).  No operand has a range limit
//   1  bf16 hi/lo  (16 significant bits, fp32 range; no longer launched:
//                  its wgrad errors measured 100x the fp32 envelope)
//   2  bf16 hi only (one MFMA: the bf16 configuration, BASELINE config #2)
// Measured against a float64 restatement of the step (tests/envelope.py):
// within ENVELOPE_K times the fp32 reference's own error.
//
// forward / dgrad  D[pixel][co] = im2col(X)[pixel][k] * Wt[k][co], with
//   k = (tap, ci) in 8-channel chunks: the block stages its input tile as an
//   NHWC image (8 channels = one 16-byte slot per pixel, pixel pitch an odd
//   number of slots so the 16 rows of an A fragment read conflict-free), so
//   an A fragment is ONE ds_read_b128 per lane (pixel, tap, 8 channels).
//   Weights are staged once per (persistent) block in fragment order.
// wgrad            D[co][n] = dY[co][pixel] * im2col(X)[pixel][n], K = pixels:
//   dY staged [co][pixel] (A: one ds_read_b128 of 8 consecutive pixels), X
//   staged NHWC and read with ds_read_b64_tr_b16, whose per-lane row address
//   absorbs the tap shift (any pixel offset, no misaligned vector reads); the
//   16 columns of an N-tile are 4 (tap, 4-channel) quads.  Bias gradients
//   are summed exactly in fp32 from the staging registers.
#include "split_common.h"

#ifndef PAIG_FWD_AUXP
#define PAIG_FWD_AUXP 1   // A/B builds: 0 = the dgrad epilogue loads its ReLU' mask when it needs it
#endif

namespace {

// ============================================================ forward / dgrad

// the fused-upsample window in the LDS of the lo image (SLA): staged, read
// by the interpolation, and overwritten by the lo pieces after a barrier (the
// interpolating threads hold them in registers meanwhile).  64 x 64 layers
// (the UNet's c15): two blocks per CU on 128-pixel tiles where the window's
// own LDS would leave one
constexpr bool sfwd_sla(bool UPS, int PM, int H, int W, int ups_bytes, int lo_bytes) {
  return UPS && PM == 0 && H * W >= 4096 && ups_bytes <= lo_bytes;
}
// bytes of LDS a forward block needs for a tile of <= tpxm pixels and ntb
// 16-channel output tiles (weights of that COUT slice + the operand images +
// the fused-upsample window)
constexpr int sfwd_lds(int CIN, int H, int W, int KS, bool UPS, int PM, int tpxm, int ntb) {
  const int CC = rup(CIN, 8) / 8, PS = CC % 2 == 0 ? CC + 1 : CC;
  const int NS = ceil_div(KS * KS * CC, 4);
  const int FPT = H * W <= tpxm ? tpxm / (H * W) : 1;
  const int RT = H * W <= tpxm ? H : rows_fit(H, W, tpxm);
  const int TWPX = W + 2 * (KS / 2);
  const int RP = W == 8 ? to_mod16(TWPX * PS, 8) : TWPX * PS;
  const int img = FPT * (RT + KS - 1) * RP * 8, wimg = NS * ntb * 64 * 8;
  const int ups = UPS ? up_window_floats(CIN, FPT, RT, W) * 4 : 0;
  return (img + wimg) * 2 * (PM == 2 ? 1 : 2) + (sfwd_sla(UPS, PM, H, W, ups, img * 2) ? 0 : ups);
}
// VGPRs per lane of a forward block (fitted to the compiler's allocation):
// accumulators, A fragments, B fragments, k-step offsets, and the staging
// registers of the next tile (prefetched); must stay within the 256 of
// 2 waves per SIMD
constexpr int sfwd_vgprs(int CIN, int H, int W, int KS, bool UPS, int tpxm, int ntb) {
  const int CC = rup(CIN, 8) / 8, NS = ceil_div(KS * KS * CC, 4);
  const int FPT = H * W <= tpxm ? tpxm / (H * W) : 1;
  const int RT = H * W <= tpxm ? H : rows_fit(H, W, tpxm);
  const int MW = ceil_div(ceil_div(FPT * RT * W, 16), 4);
  const int NL = UPS ? 1 : ceil_div(FPT * (RT + KS - 1) * (W % 2 == 0 ? W / 2 : W) * CC, 256);
  return MW * ntb * 4 + NL * 30 + ntb * 8 + NS + MW * 8 + 40;
}
// forward tile geometry, (pixels per tile) * 256 + (COUT slices): the whole
// COUT in one block on the tuned tile (256 pixels; 128 at W = 8) where that
// fits the LDS and the registers; wide layers (UNet, 48..128 channels) split
// COUT over blocks (grid.y; each slice's weights resident) and/or take
// smaller pixel tiles.  At most 4 output tiles per block.
// Pass 0 keeps two blocks per CU (LDS <= half the CU's): one 256-thread
// block is one wave per SIMD, which leaves the staging VALU work and the
// MFMAs serialised (the UNet's 32..128-channel layers: 1.2-1.7x faster).
// Not for the fused upsample (its 64 x 64 layer measured 1.2x slower on
// 64-pixel tiles).
#ifndef PAIG_FWD_UPS_TP
#define PAIG_FWD_UPS_TP 256   // A/B builds: the largest tile of the sub-64x64 fused-upsample forwards
#endif
#ifndef PAIG_FWD_TP32
#define PAIG_FWD_TP32 256     // A/B builds: the largest tile of the 32x32 forwards / dgrads (no upsample)
#endif
constexpr int sfwd_pick(int CIN, int COUT, int H, int W, int KS, bool UPS, int PM) {
  const int base = UPS && H * W < 4096 && PAIG_FWD_UPS_TP < 256   ? PAIG_FWD_UPS_TP
                   : !UPS && H * W == 1024 && PAIG_FWD_TP32 < 256 ? PAIG_FWD_TP32
                                                                  : (W == 8 ? 128 : 256);
  const int NT = ceil_div(COUT, 16);
  for (int pass = UPS && !(PM == 0 && H * W >= 4096) ? 1 : 0; pass < 3; ++pass)
    for (int nb = 1; nb <= NT; ++nb) {
      if (NT % nb != 0 || NT / nb > 4) continue;
      for (int tp = base; tp >= (pass == 1 ? base / 2 : 64); tp /= 2)
        if (sfwd_lds(CIN, H, W, KS, UPS, PM, tp, NT / nb) <= (pass == 0 ? LDS_MAX / 2 : LDS_MAX) &&
            sfwd_vgprs(CIN, H, W, KS, UPS, tp, NT / nb) <= 264 && (pass > 0 || tp >= base / 2))
          return tp * 256 + nb;
    }
  return 0;
}

template <int CIN, int COUT, int H, int W, int KS, bool UPS, int PM>
struct SFwdCfg {
  static constexpr int KK = KS * KS, PADL = KS / 2;
  static constexpr int NIMG = PM == 2 ? 1 : 2;               // hi (+ lo) images
  static constexpr int CINP = rup(CIN, 8), CC = CINP / 8;    // 8-channel chunks per pixel
  static constexpr int KC = KK * CC, NS = ceil_div(KC, 4);   // k-chunks, MFMA k-steps (4 chunks each)
  static constexpr int GEO = sfwd_pick(CIN, COUT, H, W, KS, UPS, PM);
  static_assert(GEO > 0, "no forward tile geometry fits the LDS");
  static constexpr int NB = GEO % 256;                       // COUT slices (grid.y)
  static constexpr int NT = ceil_div(COUT, 16) / NB;         // 16-channel output tiles per block
  // tile: whole rows (RT divides H) of one frame, or FPT whole frames; at
  // most TPXM pixels
  static constexpr int TPXM = GEO / 256;
  static constexpr int FPT = H * W <= TPXM ? TPXM / (H * W) : 1;
  static constexpr int RT = H * W <= TPXM ? H : rows_fit(H, W, TPXM);
  static constexpr int TPXV = FPT * RT * W;                  // valid pixels per tile
  static constexpr int NMT = ceil_div(TPXV, 16);             // M-tiles of 16 pixels
  static constexpr int MW = ceil_div(NMT, 4);                // M-tiles per wave
  static constexpr int ROWS = RT + KS - 1;
  static constexpr int TWPX = W + 2 * PADL;                  // pixel columns incl. halo
  // 16-B slots per pixel: odd, so 16 consecutive pixels hit 16 distinct
  // bank groups; an M-tile spanning two rows (W = 8) needs the row pitch
  // = 8 (mod 16) slots so the second row lands on the other 8 groups
  static constexpr int PS = CC % 2 == 0 ? CC + 1 : CC;
  static constexpr int RP = W == 8 ? to_mod16(TWPX * PS, 8) : TWPX * PS;
  static constexpr int IMG = FPT * ROWS * RP * 8;            // 16-bit elements per image
  static constexpr int WIMG = NS * NT * 64 * 8;
  static constexpr int SLB = UPS ? up_window_floats(CIN, FPT, RT, W) * 4 : 0;   // upsample window
  static constexpr bool SLA = sfwd_sla(UPS, PM, H, W, SLB, IMG * 2);
  static constexpr int LDS = (IMG + WIMG) * 2 * NIMG + (SLA ? 0 : SLB);   // incl. the upsample window
  // staging unit = UPX pixels x 8 channels, consecutive lanes on consecutive
  // pixels (coalesced loads, b128 LDS writes PS slots apart: conflict-free)
  static constexpr int UPX = W % 2 == 0 ? 2 : 1;
  static constexpr int W2 = W / UPX;
  static constexpr int NI = FPT * ROWS * W2 * CC;
  static constexpr int NL = (NI + 255) / 256;
  static constexpr bool VEC4 = W % 4 == 0;                   // 4-pixel epilogue stores stay in one row
  static_assert(H % RT == 0, "RT divides H");
  // fused 2x2 max pool of the output (flags & 64): rows are whole 16-pixel
  // M-tiles (PO per row), and a pooling kernel gives each wave MW / 2 column
  // units of row pairs (pool_mtile): its M-tile mt < MW / 2 on row 2p and
  // mt + MW / 2 on row 2p + 1, the same columns, so a lane holds both rows of
  // its windows (64-wide rows: half a row pair per wave)
  static constexpr int PO = W / 16;
  static constexpr bool POOLOK = !UPS && VEC4 && W % 16 == 0 && PO >= 1 && MW % 2 == 0 && NMT == 4 * MW &&
                                 TPXV % (2 * W) == 0 && RT % 2 == 0;
};

// aten max_pool2d's window scan (rows, then columns; a later value replaces
// the running max only if greater, or NaN), so the pooled values are
// bit-identical to maxpool_fwd_v_k's
__device__ __forceinline__ float pool4(float a, float b, float c, float d) {
  float m = a;
  if (b > m || b != b) m = b;
  if (c > m || c != c) m = c;
  if (d > m || d != d) m = d;
  return m;
}

// the window code byte of PoolOut: ReLU' bits of (a, b, c, d) = (y, x),
// (y, x+1), (y+1, x), (y+1, x+1) and the argmax in pool4's scan order
__device__ __forceinline__ unsigned char pool_code(float a, float b, float c, float d) {
  float m = a;
  int k = 0;
  if (b > m || b != b) { m = b; k = 1; }
  if (c > m || c != c) { m = c; k = 2; }
  if (d > m || d != d) { m = d; k = 3; }
  return (unsigned char)((a > 0.f ? 1 : 0) | (b > 0.f ? 2 : 0) | (c > 0.f ? 4 : 0) | (d > 0.f ? 8 : 0) | (k << 4));
}

// M-tile of wave wv's local tile mt: contiguous, or (fused pool) column unit
// u = wv MW/2 + mt % (MW/2) of row pair u / PO, top row for mt < MW/2
template <int MW, int PO, bool POOL>
__device__ __forceinline__ int fwd_mtile(int wv, int mt) {
  if constexpr (POOL) {
    constexpr int HM = MW / 2;
    const int u = wv * HM + mt % HM;
    return ((u / PO) * 2 + mt / HM) * PO + u % PO;
  } else {
    return wv * MW + mt;
  }
}

// UPT (dgrad only): the layer's input was the 2x bilinear upsample of a
// half-resolution source (blocks.py:206,219,229 feeding c9 / c12 / c15), and
// the kernel writes that SOURCE's gradient: the transposed upsample of the
// dX tile, in the epilogue.  A block walks whole frames top to bottom (its
// frames b, b + G, ...), so each half-resolution row's four full-resolution
// rows are summed in a fixed order in registers, two rows carried from one
// tile to the next; out / aux are the source's gradient and its ReLU' input
// (H/2 x W/2 planes).  Same operation order as upsample_bwd_v_k on the
// dgrad's output: bit-identical to the two-launch form.
// PF (dgrad only): the input dY is the gradient of a ReLU'd output that a 2x2
// max pool also read (the UNet's c4 / c6): the pool's backward is folded into
// the staging -- dY = ReLU'(y) * (dy + the pooled gradient at each window's
// argmax), from pout = (the pooled gradient, the forward's window codes), in
// maxpool_bwd_relu's arithmetic (conv_bwd.hip's fold)
template <int CIN, int COUT, int H, int W, int KS, bool DG, bool UPS, int PM, bool POOL = false, bool UPT = false,
          bool PF = false>
__device__ __forceinline__ void conv_fwd_split_body(FView in, FViewW out, FView aux, const float* __restrict__ w,
                                                    const float* __restrict__ bias, int F, int flags, int ntiles, XMax xm,
                                                    const s16x8* __restrict__ wp, PoolOut pout, int bx, int gx) {
  using C = SFwdCfg<CIN, COUT, H, W, KS, UPS, PM>;
  static_assert(!PF || (DG && !UPS && !POOL && !UPT && C::UPX == 2 && H % 2 == 0 && CIN % 8 == 0),
                "pool fold: dgrad staging units of one window's pixel pair");
  static_assert(!UPT || (DG && !UPS && !POOL && C::FPT == 1 && C::RT % 2 == 0 && C::VEC4 && W % 2 == 0),
                "transposed-upsample epilogue: dgrad tiles of whole row pairs");
  constexpr int KK = C::KK, CC = C::CC, KC = C::KC, NS = C::NS, NT = C::NT, MW = C::MW;
  constexpr int RT = C::RT, FPT = C::FPT, ROWS = C::ROWS, PS = C::PS, RP = C::RP;
  constexpr int NI = C::NI, NL = C::NL, PADL = C::PADL, W2 = C::W2;
  constexpr long long PLANE = UPS ? (long long)(H / 2) * (W / 2) : (long long)H * W;
  constexpr long long HW = (long long)H * W;
  extern __shared__ __attribute__((aligned(16))) short lds16[];
  short* Xh = lds16;
  short* Xl = Xh + (C::NIMG == 2 ? C::IMG : 0);
  short* Wh = lds16 + C::NIMG * C::IMG;
  short* Wl = Wh + (C::NIMG == 2 ? C::WIMG : 0);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, g = lane >> 4;
  constexpr int NRB = H / RT;
  const int co0 = blockIdx.y * NT * 16;   // this block's COUT slice
  float rmax = 0.f;                       // f16 range guard (fixed-scale A/B builds only)
  __shared__ float smax[4];

  // ---- weights in fragment order: [s][nt][lane][8]; dgrad: transposed + flipped
  auto wval = [&](int idx, int j) {
    const int ln = idx & 63, snt = idx >> 6, nt = snt % NT, s = snt / NT;
    const int kc = 4 * s + (ln >> 4), co = co0 + nt * 16 + (ln & 15);
    float v = 0.f;
    if (kc < KC && co < COUT) {
      const int tap = kc / CC, ci = (kc % CC) * 8 + j;
      if (ci < CIN) v = DG ? w[(ci * COUT + co) * KK + (KK - 1 - tap)] : w[(co * CIN + ci) * KK + tap];
    }
    return v;
  };
  // PM 0: every output channel's weights are scaled by their own power of
  // two (max |w| of the channel into [2^14, 2^15): no range limit, 22
  // significant bits), ewn[nt] for this lane's channel of N-tile nt; the
  // epilogue takes it back out exactly
  int ewn[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) ewn[nt] = 0;
  __shared__ int sew[PM == 0 ? NT * 16 : 1];   // in-kernel staging: the slice's channel exponents
  // ---- zero the halo columns (never written by the staging; again after
  // UPT's epilogue, which keeps its dX tile in the images' LDS)
  auto zero_halo = [&]() {
    if (PADL > 0) {
      for (int i = tid; i < FPT * ROWS * 2 * PADL * CC; i += 256) {
        const int cc = i % CC, hc = (i / CC) % (2 * PADL), r = i / (CC * 2 * PADL);
        const int xc = hc < PADL ? hc : W + hc;
        const int o = (r * RP + xc * PS + cc) * 8;
        *reinterpret_cast<s16x8*>(Xh + o) = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
        if (PM != 2) *reinterpret_cast<s16x8*>(Xl + o) = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
      }
    }
  };
  zero_halo();
  // ---- per-lane fragment slot offsets: pixel base per M-tile, (tap, chunk) per k-step
  int pbase[MW];
#pragma unroll
  for (int mt = 0; mt < MW; ++mt) {
    int pix = fwd_mtile<MW, C::PO, POOL>(wv, mt) * 16 + (lane & 15);
    if (pix >= C::TPXV) pix = 0;   // padding rows of the last M-tile: finite data, never stored
    const int fi = pix / (RT * W), rem = pix % (RT * W);
    pbase[mt] = (fi * ROWS + rem / W) * RP + (rem % W) * PS;
  }
  int soff[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    int kc = 4 * s + g;
    if (kc >= KC) kc = 0;   // zero weights there; read any finite slot
    const int tap = kc / CC, cc = kc % CC;
    soff[s] = (tap / KS) * RP + (tap % KS) * PS + cc;
  }

  // ---- staging: unit i = (frame fi, row r, chunk cc, pixel xp), xp fastest;
  // the next tile's loads are in flight during this tile's MFMAs
  using UP = UpStage<UPS ? CIN : 1, H, W, FPT, RT>;
  float* Sl = reinterpret_cast<float*>(C::SLA ? Xl : lds16 + C::NIMG * (C::IMG + C::WIMG));
  constexpr int UPX = C::UPX;
  // staging unit i's hi / lo pieces (both pixels) and its image offset
  auto split_px = [&](int i, const float2* v, float sc, s16x8& h0, s16x8& l0, s16x8& h1, s16x8& l1) {
    const int xp = UPX * (i % W2), r = (i / W2) % ROWS, cc = (i / (W2 * ROWS)) % CC, fi = i / (W2 * ROWS * CC);
    if constexpr (PM == 0) {
      pf32x2 sv[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) sv[c] = pf32x2{v[c].x, v[c].y} * sc;
      u32x4 a0, b0, a1, b1;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        { const HiLo q_ = split_pk(sv[2 * k].x, sv[2 * k + 1].x); a0[k] = q_.h; b0[k] = q_.l; }
        { const HiLo q_ = split_pk(sv[2 * k].y, sv[2 * k + 1].y); a1[k] = q_.h; b1[k] = q_.l; }
      }
      h0 = __builtin_bit_cast(s16x8, a0);
      l0 = __builtin_bit_cast(s16x8, b0);
      h1 = __builtin_bit_cast(s16x8, a1);
      l1 = __builtin_bit_cast(s16x8, b1);
    }
    return ((fi * ROWS + r) * RP + (xp + PADL) * PS + cc) * 8;
  };
  auto put_px = [&](int i, const float2* v, float sc) {
    const int xp = UPX * (i % W2), r = (i / W2) % ROWS, cc = (i / (W2 * ROWS)) % CC, fi = i / (W2 * ROWS * CC);
    const int o = ((fi * ROWS + r) * RP + (xp + PADL) * PS + cc) * 8;
    s16x8 h0, l0, h1, l1;
    if constexpr (PM == 0) {
      // scaled by sc (packed multiplies), split pairwise along the channels
      pf32x2 sv[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) sv[c] = pf32x2{v[c].x, v[c].y} * sc;
      u32x4 a0, b0, a1, b1;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        { const HiLo q_ = split_pk(sv[2 * k].x, sv[2 * k + 1].x); a0[k] = q_.h; b0[k] = q_.l; }
        { const HiLo q_ = split_pk(sv[2 * k].y, sv[2 * k + 1].y); a1[k] = q_.h; b1[k] = q_.l; }
      }
      h0 = __builtin_bit_cast(s16x8, a0);
      l0 = __builtin_bit_cast(s16x8, b0);
      h1 = __builtin_bit_cast(s16x8, a1);
      l1 = __builtin_bit_cast(s16x8, b1);
    } else {
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        short h, lo;
        split<PM>(v[c].x, h, lo, rmax);
        h0[c] = h;
        l0[c] = lo;
        split<PM>(v[c].y, h, lo, rmax);
        h1[c] = h;
        l1[c] = lo;
      }
    }
    *reinterpret_cast<s16x8*>(Xh + o) = h0;
    if (PM != 2) *reinterpret_cast<s16x8*>(Xl + o) = l0;
    if constexpr (UPX == 2) {
      *reinterpret_cast<s16x8*>(Xh + o + PS * 8) = h1;
      if (PM != 2) *reinterpret_cast<s16x8*>(Xl + o + PS * 8) = l1;
    }
  };
  float2 pre[UPS ? 1 : NL][8];
  // PF: each staging unit's window (8 channels): pooled gradients and codes
  float dpv[PF ? NL : 1][8];
  uint2 pcv[PF ? NL : 1];
  UP up;
  // f16 pieces (PM 0): the operand image (activations, or dgrad's gradients:
  // any magnitude) is scaled per tile by one power of two from the tile's
  // block max (tile_max, commit) and tinv takes it and the weight exponent
  // back out exactly.  The block's running max of the tile maxima goes to
  // xm.p[bx] (the wgrad of the same input scales X by their max).
  constexpr bool SCL = PM == 0, DYN = PM == 0 && PAIG_SCALE_MODE < 2;
  float tsc = 1.f, tinv[NT], xrun = 0.f;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) tinv[nt] = 1.f;
  auto tile_scale = [&]() {
    const float m = fmaxf(fmaxf(smax[0], smax[1]), fmaxf(smax[2], smax[3]));
    xrun = fmaxf(xrun, m);
    const int e = f16_scale_exp(m);
    tsc = __builtin_amdgcn_ldexpf(1.f, e);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) tinv[nt] = __builtin_amdgcn_ldexpf(1.f, -(e + ewn[nt]));
  };
  auto issue = [&](int t) {
    const int f0 = (t / NRB) * FPT, y0 = (t % NRB) * RT;
    if constexpr (UPS) {
      up.issue(in, F, f0, y0, tid);
    } else {
      // branch-free: every lane loads (out-of-tile lanes re-read the tile's
      // first pixels) and zeroes afterwards; 32-bit offsets from the tile's
      // frame (frames of one tile are fs apart: FPT > 1 only for plain views)
      const float* fb = in.frame(f0);
#pragma unroll
      for (int l = 0; l < NL; ++l) {
        const int i = tid + l * 256;
        const int xp = UPX * (i % W2), r = (i / W2) % ROWS, cc = (i / (W2 * ROWS)) % CC, fi = i / (W2 * ROWS * CC);
        const int gy = y0 + r - PADL;
        const bool ok = i < NI && f0 + fi < F && gy >= 0 && gy < H;
        const int off = fi * (int)in.fs + cc * 8 * (int)PLANE + gy * W + xp;
        static_assert(8 * PLANE <= 8 * 4096, "paig_zero_planes covers the unit");
        const float* base = ok ? fb + off : paig_zero_planes;   // one address per unit
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          // channels past CIN (CIN % 8 != 0 only) read a zero of their own
          const float* q = CIN % 8 == 0 || cc * 8 + c < CIN ? base + c * (int)PLANE : paig_zeros;
          pre[l][c] = UPX == 2 ? *reinterpret_cast<const float2*>(q) : make_float2(*q, 0.f);
        }
        if constexpr (PF) {
          constexpr int HP = H / 2, WP = W / 2;
          const int pw = (gy >> 1) * WP + (xp >> 1);
          const float* pb = ok ? pout.frame(f0) + fi * (int)pout.fs + cc * 8 * (HP * WP) + pw : paig_zero_planes;
#pragma unroll
          for (int c = 0; c < 8; ++c) dpv[l][c] = pb[c * (HP * WP)];
          const unsigned char* cb = ok ? pout.code + (long long)(f0 + fi) * pout.code_fs + ((long long)cc * HP * WP + pw) * 8
                                       : reinterpret_cast<const unsigned char*>(paig_zeros);
          pcv[l] = *reinterpret_cast<const uint2*>(cb);
        }
      }
    }
  };
  // PF: the max pool's backward on the prefetched units of tile t (before
  // their max and staging)
  auto fold = [&](int t) {
    if constexpr (PF) {
      const int y0 = (t % NRB) * RT;
#pragma unroll
      for (int l = 0; l < NL; ++l) {
        const int i = tid + l * 256;
        const int r = (i / W2) % ROWS;
        const int pr = ((y0 + r - PADL) & 1) * 2;   // window row of this unit: bits pr, pr + 1
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const unsigned b = ((c < 4 ? pcv[l].x : pcv[l].y) >> (8 * (c & 3))) & 255u;
          const int am = (int)(b >> 4) & 3;
          const float vx = pre[l][c].x + (am == pr ? dpv[l][c] : 0.f);
          const float vy = pre[l][c].y + (am == pr + 1 ? dpv[l][c] : 0.f);
          pre[l][c].x = (b >> pr) & 1u ? vx : 0.f;
          pre[l][c].y = (b >> (pr + 1)) & 1u ? vy : 0.f;
        }
      }
    }
  };
  auto commit = [&](int t) {
    if constexpr (DYN) tile_scale();
    if constexpr (UPT) zero_halo();
    if constexpr (UPS) {
      const int f0 = (t / NRB) * FPT, y0 = (t % NRB) * RT;
      up.commit(Sl, tid);
      __syncthreads();
      if constexpr (C::SLA) {
        // the window lives in the lo image's LDS: hi pieces stored now, lo
        // pieces held in registers until every thread has read the window
        static_assert(W % 4 == 0 && UPX == 2, "SLA: 4-pixel items");
        constexpr int W4 = W / 4, NIT = ceil_div(NI / 2, 256);
        s16x8 lk[NIT][4];
        int lo_off[NIT][2];
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
          const int i = tid + it * 256;
          lo_off[it][0] = -1;
          if ((NI / 2) % 256 != 0 && i >= NI / 2) break;
          const int q = i % W4, r = (i / W4) % ROWS, cc = (i / (W4 * ROWS)) % CC, fi = i / (W4 * ROWS * CC);
          const int gy = y0 + r - PADL;
          const bool ok = f0 + fi < F && gy >= 0 && gy < H;
          f32x4 o[8];
#pragma unroll
          for (int c = 0; c < 8; ++c)
            o[c] = (ok && cc * 8 + c < CIN) ? UP::row4(Sl, fi, cc * 8 + c, gy, y0, q) : f32x4{0.f, 0.f, 0.f, 0.f};
          const int ia = ((fi * CC + cc) * ROWS + r) * W2 + 2 * q;
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            float2 v[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) v[c] = make_float2(o[c][2 * u], o[c][2 * u + 1]);
            s16x8 h0, h1;
            const int off = split_px(ia + u, v, tsc, h0, lk[it][2 * u], h1, lk[it][2 * u + 1]);
            *reinterpret_cast<s16x8*>(Xh + off) = h0;
            *reinterpret_cast<s16x8*>(Xh + off + PS * 8) = h1;
            lo_off[it][u] = off;
          }
        }
        __syncthreads();   // every read of the window is done
        // the lo image's halo columns (the window overwrote them)
        for (int i = tid; i < FPT * ROWS * 2 * PADL * CC; i += 256) {
          const int cc = i % CC, hc = (i / CC) % (2 * PADL), r = i / (CC * 2 * PADL);
          const int xc = hc < PADL ? hc : W + hc;
          *reinterpret_cast<s16x8*>(Xl + (r * RP + xc * PS + cc) * 8) = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
        }
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
          if (lo_off[it][0] < 0) break;
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            *reinterpret_cast<s16x8*>(Xl + lo_off[it][u]) = lk[it][2 * u];
            *reinterpret_cast<s16x8*>(Xl + lo_off[it][u] + PS * 8) = lk[it][2 * u + 1];
          }
        }
      } else if constexpr (W % 4 == 0) {
        // units of 4 pixels x 8 channels: one row4 per channel (shared taps
        // and source reads), stored as two 2-pixel staging units
        constexpr int W4 = W / 4;
#pragma unroll 1
        for (int i = tid; i < NI / 2; i += 256) {
          const int q = i % W4, r = (i / W4) % ROWS, cc = (i / (W4 * ROWS)) % CC, fi = i / (W4 * ROWS * CC);
          const int gy = y0 + r - PADL;
          const bool ok = f0 + fi < F && gy >= 0 && gy < H;
          f32x4 o[8];
#pragma unroll
          for (int c = 0; c < 8; ++c)
            o[c] = (ok && cc * 8 + c < CIN) ? UP::row4(Sl, fi, cc * 8 + c, gy, y0, q) : f32x4{0.f, 0.f, 0.f, 0.f};
          const int ia = ((fi * CC + cc) * ROWS + r) * W2 + 2 * q;
          float2 v[8];
#pragma unroll
          for (int c = 0; c < 8; ++c) v[c] = make_float2(o[c][0], o[c][1]);
          put_px(ia, v, tsc);
#pragma unroll
          for (int c = 0; c < 8; ++c) v[c] = make_float2(o[c][2], o[c][3]);
          put_px(ia + 1, v, tsc);
        }
      } else {
#pragma unroll 1
        for (int i = tid; i < NI; i += 256) {
          const int xp = UPX * (i % W2), r = (i / W2) % ROWS, cc = (i / (W2 * ROWS)) % CC, fi = i / (W2 * ROWS * CC);
          const int gy = y0 + r - PADL;
          const bool ok = f0 + fi < F && gy >= 0 && gy < H;
          float2 v[8];
#pragma unroll
          for (int c = 0; c < 8; ++c)
            v[c] = (ok && cc * 8 + c < CIN)
                       ? make_float2(UP::px1(Sl, fi, cc * 8 + c, gy, y0, xp),
                                     UPX == 2 ? UP::px1(Sl, fi, cc * 8 + c, gy, y0, xp + 1) : 0.f)
                       : make_float2(0.f, 0.f);
          put_px(i, v, tsc);
        }
      }
    } else {
#pragma unroll
      for (int l = 0; l < NL; ++l) {
        const int i = tid + l * 256;
        if (NI % 256 != 0 && i >= NI) break;
        put_px(i, pre[l], tsc);
      }
    }
  };

  // PM 0: this wave's max |operand| of the prefetched tile into smax[wv],
  // before the loop-top barrier (commit reads it after; the previous tile's
  // reads finished before the post-commit barrier)
  auto tile_max = [&]() {
    float m = 0.f;
    if constexpr (UPS) {
      m = up.amax();   // the window bounds its upsampled values
    } else {
#pragma unroll
      for (int l = 0; l < NL; ++l)
#pragma unroll
        for (int c = 0; c < 8; ++c) m = amax2(m, pre[l][c].x, pre[l][c].y);
    }
    m = wave_max_u(m);
    if (lane == 0) smax[wv] = m;
  };

  // logical tile lt; xcd_tile() gives the physical one; past the last tile,
  // tile ntiles lies beyond frame F and every lane reads paig_zeros (the
  // prefetch stays unconditional: branch-free for the load counting)
  // UPT: logical tile l of this block is band l % NRB of its (l / NRB)-th frame
  int lt = UPT ? 0 : bx;
  const int lstep = UPT ? 1 : gx;
  auto tile_of = [&](int l) {
    if constexpr (UPT) {
      const int f = bx + (l / NRB) * gx;
      return f < F ? f * NRB + l % NRB : ntiles;
    } else {
      return l < ntiles ? xcd_tile(l, ntiles) : ntiles;
    }
  };
  issue(tile_of(lt));
  if (PM == 0 && wp != nullptr) {
    // pre-split images of the whole COUT (paig_conv_wprep, once per step):
    // the channel exponents (header), then this slice's NT tiles of every
    // k-step, coalesced 16-byte copies
    constexpr int NTT = NT * C::NB, WLO = NS * NTT * 64, HDR = NTT * 16 * 4 / 16;
    const int* hdr = reinterpret_cast<const int*>(wp);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) ewn[nt] = hdr[co0 + nt * 16 + (lane & 15)];
    const s16x8* img = wp + HDR;
    for (int idx = tid; idx < NS * NT * 64; idx += 256) {
      const int s = idx / (NT * 64), r = idx - s * (NT * 64);
      const int src = (s * NTT + blockIdx.y * NT) * 64 + r;
      *reinterpret_cast<s16x8*>(Wh + idx * 8) = img[src];
      *reinterpret_cast<s16x8*>(Wl + idx * 8) = img[WLO + src];
    }
  } else {
    if constexpr (PM == 0) {
      // the slice's channel maxima (bit patterns of non-negative floats
      // order as integers: an LDS atomic max, order-independent)
      for (int i = tid; i < NT * 16; i += 256) sew[i] = 0;
      __syncthreads();
      float pm[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) pm[nt] = 0.f;
      for (int idx = tid; idx < NS * NT * 64; idx += 256) {
        const int nt = (idx >> 6) % NT;
#pragma unroll
        for (int j = 0; j < 8; ++j) pm[nt] = fmaxf(pm[nt], fabsf(wval(idx, j)));
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) atomicMax(&sew[nt * 16 + (tid & 15)], __builtin_bit_cast(int, pm[nt]));
      __syncthreads();
      for (int i = tid; i < NT * 16; i += 256) sew[i] = f16_scale_exp_v(__builtin_bit_cast(float, sew[i]));
      __syncthreads();
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) ewn[nt] = sew[nt * 16 + (lane & 15)];
    }
    for (int idx = tid; idx < NS * NT * 64; idx += 256) {
      const int cl = ((idx >> 6) % NT) * 16 + (idx & 15);
      const int e = PM == 0 ? sew[cl] : 0;
      s16x8 vh, vl;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        short h, l;
        split<PM>(__builtin_amdgcn_ldexpf(wval(idx, j), e), h, l, rmax);
        vh[j] = h;
        vl[j] = l;
      }
      *reinterpret_cast<s16x8*>(Wh + idx * 8) = vh;
      if (PM != 2) *reinterpret_cast<s16x8*>(Wl + idx * 8) = vl;
    }
  }
  if constexpr (!DYN) {   // fixed activation scale (A/B builds): the weight exponents alone
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) tinv[nt] = __builtin_amdgcn_ldexpf(1.f, -ewn[nt]);
  }
  // the bias of this lane's output channels (block constant)
  float bvs[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int co = co0 + nt * 16 + (lane & 15);
    bvs[nt] = *(bias && co < COUT ? bias + co : paig_zeros);
    asm volatile("" ::"v"(bvs[nt]));   // arrived before the loop: no wait on it behind a prefetch
  }
  // UPT: this thread's items (channel, source column) and their carried
  // partial sums of source rows kB (the tile's last) and kB + 1
  constexpr int WS2 = W / 2, NCL = NT * 16, NUI = UPT ? ceil_div(NCL * WS2, 256) : 1;
  float car0[NUI], car1[NUI];
  float auxu[UPT ? NUI : 1][UPT ? RT / 2 + 1 : 1];   // ReLU' inputs of the rows the tile completes
  // loaded before the tile's MFMAs (their latency hides behind them)
  auto upt_aux = [&](int tile) {
    if constexpr (UPT) {
      if (flags & 2) {
        const int f = tile / NRB, kA = (tile % NRB) * (RT / 2);
#pragma unroll
        for (int u = 0; u < NUI; ++u) {
          const int item = tid + u * 256;
          const int cl = item / WS2, j = item % WS2;
          const bool ok = (NCL * WS2) % 256 == 0 || item < NCL * WS2;
#pragma unroll
          for (int i = 0; i <= RT / 2; ++i) {
            const int k = kA - 1 + i;
            const float* ap = aux.frame(f) + (long long)(co0 + cl) * ((H / 2) * WS2) + (long long)k * WS2 + j;
            auxu[u][i] = *(ok && k >= 0 && k < H / 2 ? ap : paig_zeros);
          }
        }
      }
    }
  };
  auto upt_epilogue = [&](int tile, f32x4 (&a)[MW][NT]) {
    constexpr int HS = H / 2, KR = RT / 2 + 2;   // P[i]: source row kA - 1 + i
    static_assert(!UPT || RT * NCL * W * 4 <= C::NIMG * C::IMG * 2, "the dX tile fits the image's LDS");
    const int f = tile / NRB, band = tile % NRB, kA = band * (RT / 2);
    __syncthreads();   // every wave's fragment reads of the image are done
    float* RB = reinterpret_cast<float*>(lds16);   // the dX tile, [row][channel][x]
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int cl = nt * 16 + (lane & 15);
#pragma unroll
      for (int mt = 0; mt < MW; ++mt) {
        const int pix = fwd_mtile<MW, C::PO, false>(wv, mt) * 16 + (lane >> 4) * 4;
        if (pix >= C::TPXV) continue;
        f32x4 v = a[mt][nt];
        if constexpr (SCL) v *= tinv[nt];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += bvs[nt];
        *reinterpret_cast<f32x4*>(RB + ((pix / W) * NCL + cl) * W + pix % W) = v;
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NUI; ++u) {
      const int item = tid + u * 256;
      if ((NCL * WS2) % 256 != 0 && item >= NCL * WS2) break;
      const int cl = item / WS2, j = item % WS2, co = co0 + cl;
      float P[KR];
      P[0] = band == 0 ? 0.f : car0[u];
      P[1] = band == 0 ? 0.f : car1[u];
#pragma unroll
      for (int i = 2; i < KR; ++i) P[i] = 0.f;
      // upsample_bwd_v_k's taps and order: each full row's columns 2j-1 ..
      // 2j+2, then the rows 2k-1 .. 2k+2 of source row k in increasing order
      const float wxa = j >= 1 ? 0.25f : 0.f, wxb = j == 0 ? 1.f : 0.75f;
      const float wxc = j == WS2 - 1 ? 1.f : 0.75f, wxd = j <= WS2 - 2 ? 0.25f : 0.f;
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        const float* rp = RB + (r * NCL + cl) * W + 2 * j;
        const float2 m2 = *reinterpret_cast<const float2*>(rp);
        float hs = 0.f;
        if (wxa != 0.f) hs = fmaf(wxa, rp[-1], hs);
        hs = fmaf(wxb, m2.x, hs);
        hs = fmaf(wxc, m2.y, hs);
        if (wxd != 0.f) hs = fmaf(wxd, rp[2], hs);
        const int m = kA + r / 2;   // full row 2m (r even) or 2m + 1 (r odd)
        if (r % 2 == 0) {
          if (m >= 1) P[r / 2] = fmaf(0.25f, hs, P[r / 2]);                 // row 2k+2 of k = m - 1
          P[r / 2 + 1] = fmaf(m == 0 ? 1.f : 0.75f, hs, P[r / 2 + 1]);      // row 2k of k = m
        } else {
          P[r / 2 + 1] = fmaf(m == HS - 1 ? 1.f : 0.75f, hs, P[r / 2 + 1]);  // row 2k+1 of k = m
          if (m + 1 <= HS - 1) P[r / 2 + 2] = fmaf(0.25f, hs, P[r / 2 + 2]);  // row 2k-1 of k = m + 1
        }
      }
      // complete: rows kA - 1 .. kB - 1, and kB on the frame's last band
      const bool last = band == NRB - 1;
      const long long po = (long long)co * (HS * WS2) + j;
#pragma unroll
      for (int i = 0; i <= RT / 2; ++i) {
        const int k = kA - 1 + i;
        if (k < 0 || (i == RT / 2 && !last)) continue;
        float v = P[i];
        if (flags & 2) v = auxu[u][i] > 0.f ? v : 0.f;
        out.frame(f)[po + k * WS2] = v;
      }
      car0[u] = P[RT / 2];
      car1[u] = P[RT / 2 + 1];
    }
  };
  for (;; lt += lstep) {
    const int tile = tile_of(lt);
    if (tile >= ntiles) break;
    const int f0 = (tile / NRB) * FPT, y0 = (tile % NRB) * RT;
    fold(tile);
    if constexpr (DYN) tile_max();
    __syncthreads();   // previous tile's fragment reads are done
    commit(tile);
    __syncthreads();
    // dgrad: this tile's ReLU' mask for the epilogue (AUXP), loaded before the
    // next tile's prefetch so that its latency hides behind the MFMAs
    constexpr bool AUXP = PAIG_FWD_AUXP && DG && C::VEC4 && !POOL && !UPT && MW * NT <= 8;
    f32x4 auxv[AUXP ? MW : 1][AUXP ? NT : 1];
    if constexpr (AUXP) {
      if (flags & 2) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const int co = co0 + nt * 16 + (lane & 15);
#pragma unroll
          for (int mt = 0; mt < MW; ++mt) {
            const int pix = fwd_mtile<MW, C::PO, POOL>(wv, mt) * 16 + (lane >> 4) * 4;
            const int fi = pix / (RT * W), rem = pix % (RT * W);
            const int f = f0 + fi;
            const bool ok = co < COUT && pix < C::TPXV && f < F;
            const float* ap = ok ? aux.frame(f) + co * HW + (long long)(y0 + rem / W) * W + rem % W : paig_zero_planes;
            auxv[mt][nt] = *reinterpret_cast<const f32x4*>(ap);
          }
        }
      }
    }
    upt_aux(tile);
    issue(tile_of(lt + lstep));
    f32x4 acc[MW][NT];
#pragma unroll
    for (int mt = 0; mt < MW; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      s16x8 bh[NT], bl[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int o = ((s * NT + nt) * 64 + lane) * 8;
        bh[nt] = *reinterpret_cast<const s16x8*>(Wh + o);
        bl[nt] = PM != 2 ? *reinterpret_cast<const s16x8*>(Wl + o) : bh[nt];
      }
#pragma unroll
      for (int mt = 0; mt < MW; ++mt) {
        const int o = (pbase[mt] + soff[s]) * 8;
        const s16x8 ah = *reinterpret_cast<const s16x8*>(Xh + o);
        const s16x8 al = PM != 2 ? *reinterpret_cast<const s16x8*>(Xl + o) : ah;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mma3<PM>(ah, al, bh[nt], bl[nt], acc[mt][nt]);
      }
    }
    if constexpr (UPT) {
      upt_epilogue(tile, acc);
      continue;
    }
    // ---- epilogue: lane holds pixels (lane>>4)*4 + r of each M-tile for co = nt*16 + (lane&15)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int co = co0 + nt * 16 + (lane & 15);
      if (co >= COUT) continue;
      const float bv = bvs[nt];
      f32x4 vv[MW];   // the stored values (fused pool)
#pragma unroll
      for (int mt = 0; mt < MW; ++mt) {
        const int pix = fwd_mtile<MW, C::PO, POOL>(wv, mt) * 16 + (lane >> 4) * 4;
        if constexpr (C::VEC4) {
          // 4 pixels of one row (rows hold a multiple of 4 pixels)
          if (pix >= C::TPXV) continue;
          const int fi = pix / (RT * W), rem = pix % (RT * W);
          const int y = y0 + rem / W, x = rem % W, f = f0 + fi;
          if (f >= F) continue;
          float* op = out.frame(f) + co * HW + (long long)y * W + x;
          f32x4 v = acc[mt][nt];
          if constexpr (SCL) v *= tinv[nt];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += bv;
          if (flags & 1) {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = v[r] < 0.f ? 0.f : v[r];
          }
          if (flags & 4) v += *reinterpret_cast<const f32x4*>(op);
          if (flags & 2) {
            f32x4 m;
            if constexpr (AUXP) m = auxv[mt][nt];
            else m = *reinterpret_cast<const f32x4*>(aux.frame(f) + co * HW + (long long)y * W + x);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = m[r] > 0.f ? v[r] : 0.f;
          }
          *reinterpret_cast<f32x4*>(op) = v;
          if constexpr (POOL) vv[mt] = v;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int pr = pix + r;
            if (pr >= C::TPXV) break;
            const int fi = pr / (RT * W), rem = pr % (RT * W);
            const int y = y0 + rem / W, x = rem % W, f = f0 + fi;
            if (f >= F) continue;
            float* op = out.frame(f) + co * HW + (long long)y * W + x;
            float v = (SCL ? acc[mt][nt][r] * tinv[nt] : acc[mt][nt][r]) + bv;
            if (flags & 1) v = v < 0.f ? 0.f : v;
            if (flags & 4) v += *op;
            if (flags & 2) v = aux.frame(f)[co * HW + (long long)y * W + x] > 0.f ? v : 0.f;
            *op = v;
          }
        }
      }
      if constexpr (POOL) {
        {
          // rows y (local M-tile mt) and y + 1 (mt + MW/2) -> pooled row y / 2,
          // columns x/2, x/2 + 1
#pragma unroll
          for (int mt = 0; mt < MW / 2; ++mt) {
            const int pix = fwd_mtile<MW, C::PO, POOL>(wv, mt) * 16 + (lane >> 4) * 4;
            if (pix >= C::TPXV) continue;
            const int fi = pix / (RT * W), rem = pix % (RT * W);
            const int y = y0 + rem / W, x = rem % W, f = f0 + fi;
            if (f >= F) continue;
            const f32x4 a = vv[mt], b = vv[mt + MW / 2];
            const float2 o = make_float2(pool4(a[0], a[1], b[0], b[1]), pool4(a[2], a[3], b[2], b[3]));
            *reinterpret_cast<float2*>(pout.frame(f) + (long long)co * (HW / 4) + (y / 2) * (W / 2) + x / 2) = o;
            if (pout.code) {   // the two windows' codes (PoolOut): ReLU' bits + argmax
              unsigned char* cp = pout.code + (long long)f * pout.code_fs +
                                  (((long long)(co >> 3) * (H / 2) + y / 2) * (W / 2) + x / 2) * 8 + (co & 7);
              cp[0] = pool_code(a[0], a[1], b[0], b[1]);
              cp[8] = pool_code(a[2], a[3], b[2], b[3]);
            }
          }
        }
      }
    }
  }
  if constexpr (PM == 0) {
    f16_range_note(rmax);
    if (xm.p && blockIdx.y == 0) {
      if (tid == 0) xm.p[bx] = xrun;
      if (bx == 0)
        for (int i = gx + tid; i < xm.n; i += 256) xm.p[i] = 0.f;
      for (int i = bx * 256 + tid; i < xm.zn; i += gx * 256) xm.z[i] = 0.f;   // later layers' slots
    }
  }
}

// bx / gx: this block's index and the block count of the tile walk (the
// launch's own, or those of the forward's share of a merged launch)
template <int CIN, int COUT, int H, int W, int KS, bool DG, bool UPS, int PM, bool POOL = false, bool UPT = false,
          bool PF = false>
__global__ void __launch_bounds__(256, 2)
conv_fwd_split_k(FView in, FViewW out, FView aux, const float* __restrict__ w, const float* __restrict__ bias, int F,
                 int flags, int ntiles, XMax xm, const s16x8* __restrict__ wp, PoolOut pout) {
  conv_fwd_split_body<CIN, COUT, H, W, KS, DG, UPS, PM, POOL, UPT, PF>(in, out, aux, w, bias, F, flags, ntiles, xm, wp,
                                                                      pout, blockIdx.x, gridDim.x);
}

// ===================================================================== wgrad
#ifndef PAIG_WG_UPS_OB
#define PAIG_WG_UPS_OB 32
#endif

#ifndef PAIG_WG_SLA
#define PAIG_WG_SLA 0   // A/B builds: 1 = the 64x64 fused-upsample wgrad's window in the lo X image's LDS,
#endif                  // two blocks per CU on 16-channel output slices (mnist within noise: 18.63 vs 18.66 ms)
// waves splitting the N-tiles: as few as keep <= 40 accumulators per lane
constexpr int swg_wn(int MT, int NT) { return MT * NT * 4 <= 40 ? 1 : (MT * ceil_div(NT, 2) * 4 <= 40 ? 2 : 4); }
// the fused-upsample window in the lo X image's LDS (as the forward's SLA):
// 64 x 64 layers (mnist c15), two blocks per CU on 16-output-channel slices
constexpr bool swg_sla(bool UPS, int PM, int H, int W, int win_bytes, int xlo_bytes) {
  return PAIG_WG_SLA && UPS && PM == 0 && H * W >= 4096 && win_bytes <= xlo_bytes;
}
// LDS of a wgrad block staging CINB input and COUTB output-gradient channels
constexpr int swg_lds(int CINB, int COUTB, int H, int W, int KS, bool UPS, int PM) {
  const int CQ = rup(CINB, 4) / 4, FPT = H * W <= 256 ? 256 / (H * W) : 1;
  const int RT = H * W <= 256 ? H : rows_fit(H, W, 256);
  const int TWPX = W + 2 * (KS / 2 > 0 ? 2 : 0);
  const int XPL = rup(FPT * (RT + KS - 1) * TWPX * 4 + 80, 128);
  const int win = UPS ? up_window_floats(CINB, FPT, RT, W) * 4 : 0;
  const int stg = (CQ * XPL + COUTB * 264) * 2 * (PM == 2 ? 1 : 2) +
                  (swg_sla(UPS, PM, H, W, win, CQ * XPL * 2) ? 0 : win);
  const int MT = ceil_div(COUTB, 16), NT = ceil_div(KS * KS * CQ, 4);
  const int red = 4 * MT * ceil_div(NT, swg_wn(MT, NT)) * 4 * 64 * 4;
  return stg > red ? stg : red;
}
// channel slices of a wgrad block, CINB * 4096 + COUTB: the block reduces the
// gradient of CINB input x COUTB output channels (grid.y, grid.z) over its
// pixel tiles.  The whole layer where its accumulators (4 waves splitting N)
// and staging fit; wide layers take the slice with the most work per block.
constexpr int swg_pick(int CIN, int COUT, int H, int W, int KS, bool UPS, int PM) {
  const int ci[] = {CIN, 128, 64, 32, 16, 8}, oc[] = {COUT, 128, 64, 32, 16};
  // pass 0: two blocks per CU (see sfwd_pick; not for the 64 x 64 fused
  // upsample, whose halved channel slices measured 4% slower)
  for (int pass = UPS && H * W >= 4096 && !(PM == 0 && PAIG_WG_SLA) ? 1 : 0; pass < 2; ++pass) {
    int best = 0, bw = 0, bs = 0;
    for (int cb : ci) {
      if (cb > CIN || CIN % cb != 0 || (cb != CIN && cb % 4 != 0)) continue;
      for (int ob : oc) {
        if (ob > COUT || COUT % ob != 0 || (UPS && ob > (pass ? PAIG_WG_UPS_OB : 16))) continue;   // UPS: dY staging registers
        const int MT = ceil_div(ob, 16), NT = ceil_div(KS * KS * ceil_div(cb, 4), 4);
        if (MT * ceil_div(NT, 4) * 4 > 40 || swg_lds(cb, ob, H, W, KS, UPS, PM) > (pass == 0 ? LDS_MAX / 2 : LDS_MAX))
          continue;
        // ties: the fewest staged channels
        const int sc = cb + ob;
        if (cb * ob > bw || (cb * ob == bw && sc < bs)) {
          bw = cb * ob;
          bs = sc;
          best = cb * 4096 + ob;
        }
      }
    }
    if (best) return best;
  }
  return 0;
}

template <int CIN, int COUT, int H, int W, int KS, bool UPS, int PM>
struct SWgCfg {
  static constexpr int KK = KS * KS, PADL = KS / 2;
  static constexpr int NIMG = PM == 2 ? 1 : 2;
  static constexpr int SLC = swg_pick(CIN, COUT, H, W, KS, UPS, PM);
  static_assert(SLC > 0, "no wgrad channel slice fits");
  static constexpr int CINB = SLC / 4096, COUTB = SLC % 4096;  // channels per block
  static constexpr int NSI = CIN / CINB, NSO = COUT / COUTB;   // slices (grid.y, grid.z)
  static constexpr int CINQ = rup(CINB, 4), CQ = CINQ / 4;    // 4-channel quads per pixel
  static constexpr int NQ = KK * CQ;                          // (tap, quad) column quads
  static constexpr int NT = ceil_div(NQ, 4);                  // N-tiles of 16 columns
  static constexpr int NCOL = CIN * KK;                       // slab row: the whole layer
  static constexpr int MT = ceil_div(COUTB, 16), COP = MT * 16;
  static constexpr int WN = swg_wn(MT, NT);
  static constexpr int WP = 4 / WN, NTW = ceil_div(NT, WN);
  // tile: whole rows (RT divides H) of one frame or FPT whole frames, <= 256
  // pixels; k-blocks of 32 tile pixels (the last one zero-padded in dY)
  static constexpr int TPX = 256;
  static constexpr int FPT = H * W <= TPX ? TPX / (H * W) : 1;
  static constexpr int RT = H * W <= TPX ? H : rows_fit(H, W, TPX);
  static constexpr int TPXV = FPT * RT * W;                   // valid pixels per tile
  static constexpr int KB = ceil_div(TPXV, 32);               // k-blocks of 32 pixels per tile
  // FAST: every k-block is 32 pixels of whole rows of one frame, so a lane's
  // transposed-read rows are a fixed offset from the k-block base
  static constexpr bool FAST = TPXV == 256 && (RT * W) % 32 == 0 && (W % 32 == 0 || 32 % W == 0);
  static constexpr int ROWS = RT + KS - 1;
  // input column x sits at image column x + OFFX: even, so a 2-pixel staging
  // unit is one aligned 16-B write per plane
  static constexpr int OFFX = PADL > 0 ? 2 : 0;
  static constexpr int TWPX = W + 2 * OFFX;
  // X image: one plane per 4-channel quad, [pixel position][4] (8 B per pixel)
  // so the staging writes of consecutive pixels are consecutive; plane bases
  // are 256-B aligned plus {0, 32, 128, 160} B so the transposed reads of an
  // N-tile's 4 quads (4 pixels x 2 lane groups each) fill distinct banks
  static constexpr int XPL = rup(FPT * ROWS * TWPX * 4 + 80, 128);   // room for the <= 80-element offset
  static constexpr int XIMG = CQ * XPL;
  static constexpr int DP = TPX + 8;                          // dY row pitch: 16 rows -> 16 bank groups
  static constexpr int DIMG = COUTB * DP;   // rows co >= COUTB of an A fragment re-read rows co % COUTB
  static constexpr int STG = (XIMG + DIMG) * 2 * NIMG;
  static constexpr bool SLA = swg_sla(UPS, PM, H, W, UPS ? up_window_floats(CINB, FPT, RT, W) * 4 : 0, XIMG * 2);
  static constexpr int RED = 4 * MT * NTW * 4 * 64 * 4;
  static constexpr int LDS = STG > RED ? STG : RED;
  static constexpr int UPX = W % 2 == 0 ? 2 : 1;              // X units: UPX pixels x 4 channels
  static constexpr int W2 = W / UPX;
  static constexpr int NIX = FPT * ROWS * W2 * CQ, NLX = (NIX + 255) / 256;
  // dY units: DU pixels (of one row) x 1 channel; 3 for 3bp's 9 x 9 level
  // (1-pixel units there need 31 units per thread, and as many bias partial
  // registers: the kernel spilled 88 VGPRs)
  static constexpr int DU = W % 4 == 0 ? 4 : (W % 2 == 0 ? 2 : (W % 3 == 0 ? 3 : 1));
  static constexpr int NPU = TPXV / DU;                       // dY units per channel
  static constexpr int NID = COUTB * NPU, NLD = (NID + 255) / 256;
  static constexpr int SLAB = COUT * NCOL + COUT;
  // waves per SIMD the registers must allow: 3 where three blocks fit the LDS
  // (narrow whole-layer blocks only: the 32-wide / channel-sliced ones need
  // more than the 168 registers of 3 waves)
  static constexpr int MINW =
      2 * LDS > 160 * 1024 ? 1
      : 3 * LDS <= 160 * 1024 && NSI * NSO == 1 && (CIN <= 24 || (UPS && COUT <= 16)) && !(MT == 2 && FPT > 1) ? 3 : 2;
  static_assert(H % RT == 0, "RT divides H");
  static_assert(TPXV % DU == 0, "dY units");
};

// PF: dY is the gradient of a ReLU'd output that a 2x2 max pool also read
// (the UNet's c4 / c6, blocks.py:186-197): the pool's backward is folded into
// the dY staging -- dY = ReLU'(y) * (dy + the pooled gradient pin at each
// window's argmax), from the window codes the forward's fused pool wrote
// (paig_conv2d_fwd_pwc), in maxpool_bwd_relu's arithmetic
template <int CIN, int COUT, int H, int W, int KS, bool UPS, int PM, bool PF = false>
__global__ void __launch_bounds__(256, (SWgCfg<CIN, COUT, H, W, KS, UPS, PM>::MINW))
conv_wgrad_split_k(FView x_, FView dy_, float* __restrict__ slab, int F, int ntiles, XMax xm, PoolOut pin) {
  using C = SWgCfg<CIN, COUT, H, W, KS, UPS, PM>;
  static_assert(!PF || (!UPS && C::DU == 4 && C::FPT == 1 && W % 4 == 0 && H % 2 == 0), "pool fold: 4-pixel dY units");
  constexpr int CINB = C::CINB, COUTB = C::COUTB;
  constexpr int KK = C::KK, CQ = C::CQ, NQ = C::NQ, NT = C::NT, NCOL = C::NCOL, MT = C::MT, COP = C::COP;
  constexpr int WN = C::WN, WP = C::WP, NTW = C::NTW, RT = C::RT, FPT = C::FPT, ROWS = C::ROWS;
  constexpr int TWPX = C::TWPX, XPL = C::XPL, DP = C::DP, KB = C::KB, PADL = C::PADL, OFFX = C::OFFX, W2 = C::W2;
  constexpr int UPX = C::UPX, DU = C::DU, NPU = C::NPU, TPXV = C::TPXV;
  constexpr int NIX = C::NIX, NLX = C::NLX, NID = C::NID, NLD = C::NLD;
  constexpr long long PLANE = UPS ? (long long)(H / 2) * (W / 2) : (long long)H * W;
  constexpr long long HW = (long long)H * W;
  // this block's channel slice: input channels ci0.., output channels co0..
  const int ci0 = blockIdx.y * CINB, co0 = blockIdx.z * COUTB;
  FView x = x_, dy = dy_;
  x.p += ci0 * PLANE;
  dy.p += co0 * HW;
  extern __shared__ __attribute__((aligned(16))) short lds16[];
  short* Xh = lds16;
  short* Xl = Xh + (C::NIMG == 2 ? C::XIMG : 0);
  short* Dh = lds16 + C::NIMG * C::XIMG;
  short* Dl = Dh + (C::NIMG == 2 ? C::DIMG : 0);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, g = lane >> 4;
  const int wn = wv % WN, wp = wv / WN;
  constexpr int NRB = H / RT;
  // PM 0 (f16 pieces): X (activations) scaled by one power of two for the
  // whole launch, from the max |X| the forward conv of the same input
  // recorded per block (xm; without it the fixed 2^PAIG_A_EXP, range-
  // guarded); dY (gradients, any magnitude) scaled by a running power of two
  // 2^ecd: a tile's block-wide max |dY| gives the exponent that puts it in
  // [2^14, 2^15); when a tile needs a smaller one than the running exponent,
  // the accumulators (held at scale 2^(ecx + ecd)) are rescaled first,
  // exactly.  Every element then keeps 22 significant bits or an absolute
  // error below 2^-40 of its operand's largest (bf16 pieces keep 16 bits; an
  // unscaled f16 lo piece goes subnormal below |v| = 1/8).
  int ecx = PAIG_A_EXP;
  float xsc = 1.f;   // 2^ecx, set before the first tile
  int ecd = PAIG_SCALE_MODE < 2 ? 100 : 0;
  float dsc = __builtin_amdgcn_ldexpf(1.f, ecd);
  float rmax = 0.f;   // range guard of the scaled activations
  __shared__ float smax[4];

  auto xplane = [](int cq) { return cq * XPL + ((cq & 1) ? 16 : 0) + ((cq & 2) ? 64 : 0); };
  // ---- zero the halo columns of X (never staged)
  if (OFFX > 0) {
    for (int i = tid; i < FPT * ROWS * 2 * OFFX; i += 256) {
      const int hc = i % (2 * OFFX), r = i / (2 * OFFX);
      const int xc = hc < OFFX ? hc : W + hc;
      for (int cq = 0; cq < CQ; ++cq) {
        *reinterpret_cast<s16x4*>(Xh + xplane(cq) + (r * TWPX + xc) * 4) = s16x4{0, 0, 0, 0};
        if (PM != 2) *reinterpret_cast<s16x4*>(Xl + xplane(cq) + (r * TWPX + xc) * 4) = s16x4{0, 0, 0, 0};
      }
    }
  }
  // padded pixels of the last k-block: dY = 0 (never staged)
  if (KB * 32 > TPXV) {
    for (int i = tid; i < COUTB * (KB * 32 - TPXV); i += 256) {
      const int co = i / (KB * 32 - TPXV), pt = TPXV + i % (KB * 32 - TPXV);
      Dh[co * DP + pt] = 0;
      if (PM != 2) Dl[co * DP + pt] = 0;
    }
  }
  // ---- per-lane transposed-read addressing. Lane 4q+p of its 16-lane group
  // supplies row q (pixel 8g + 4h + q of the k-block) of column quad p.
  const int qq = (lane >> 2) & 3, pp = lane & 3;
  int roff[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int j = 8 * g + 4 * h + qq;
    roff[h] = (j / W) * TWPX + j % W + (OFFX - PADL);
  }
  int colt[NTW];
#pragma unroll
  for (int jn = 0; jn < NTW; ++jn) {
    int cq = (wn + jn * WN) * 4 + pp;
    if (cq >= NQ) cq = 0;   // padded columns: any finite data, never stored
    const int tap = cq / CQ, ciq = cq % CQ;
    colt[jn] = xplane(ciq) + ((tap / KS) * TWPX + tap % KS) * 4;
  }
  f32x4 acc[MT][NTW];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[m][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc[NLD];
#pragma unroll
  for (int l = 0; l < NLD; ++l) bacc[l] = 0.f;

  // X units (1 pixel x 4 channels, pixel fastest) are prefetched a tile
  // ahead where their registers are cheap, else loaded synchronously; fused-
  // upsample inputs go through UpStage (half-resolution window, prefetched).
  using UP = UpStage<UPS ? CINB : 1, H, W, FPT, RT>;
  float* Sl = reinterpret_cast<float*>(C::SLA ? Xl : lds16 + C::NIMG * (C::XIMG + C::DIMG));
  constexpr bool XPIPE = !UPS && NLX * 8 + NLD * 4 <= (C::MINW == 3 ? 24 : 48);
  auto load_x = [&](int t, int i, float2* v) {   // branch-free, 32-bit offsets (see the forward kernel)
    const int f0 = (t / NRB) * FPT, y0 = (t % NRB) * RT;
    const int xp = UPX * (i % W2), r = (i / W2) % ROWS, cq = (i / (W2 * ROWS)) % CQ, fi = i / (W2 * ROWS * CQ);
    const int gy = y0 + r - PADL;
    const bool ok = i < NIX && f0 + fi < F && gy >= 0 && gy < H;
    const float* fb = x.frame(f0);
    const int off = fi * (int)x.fs + cq * 4 * (int)PLANE + gy * W + xp;
    const float* base = ok ? fb + off : paig_zero_planes;   // one address per unit
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float* q = CINB % 4 == 0 || cq * 4 + c < CINB ? base + c * (int)PLANE : paig_zeros;
      v[c] = UPX == 2 ? *reinterpret_cast<const float2*>(q) : make_float2(*q, 0.f);
    }
  };
  // SLA: store unit i's hi pieces only; its lo pieces and offset come back
  auto put_x = [&](int i, const float2* v, s16x8* keep_lo = nullptr, int* keep_o = nullptr) {
    const int xp = UPX * (i % W2), r = (i / W2) % ROWS, cq = (i / (W2 * ROWS)) % CQ, fi = i / (W2 * ROWS * CQ);
    const int o = xplane(cq) + ((fi * ROWS + r) * TWPX + xp + OFFX) * 4;
    s16x8 hv, lv;
    if constexpr (PM == 0) {
      pf32x2 sv[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        sv[c] = pf32x2{v[c].x, v[c].y} * xsc;
        rmax = amax2(rmax, sv[c].x, sv[c].y);
      }
      u32x4 a, b;
      { const HiLo q_ = split_pk(sv[0].x, sv[1].x); a[0] = q_.h; b[0] = q_.l; }
      { const HiLo q_ = split_pk(sv[2].x, sv[3].x); a[1] = q_.h; b[1] = q_.l; }
      { const HiLo q_ = split_pk(sv[0].y, sv[1].y); a[2] = q_.h; b[2] = q_.l; }
      { const HiLo q_ = split_pk(sv[2].y, sv[3].y); a[3] = q_.h; b[3] = q_.l; }
      hv = __builtin_bit_cast(s16x8, a);
      lv = __builtin_bit_cast(s16x8, b);
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        short h, lo;
        split<PM>(v[c].x, h, lo, rmax);
        hv[c] = h;
        lv[c] = lo;
        split<PM>(v[c].y, h, lo, rmax);
        hv[4 + c] = h;
        lv[4 + c] = lo;
      }
    }
    if (keep_lo) {   // (SLA: UPX == 2)
      *reinterpret_cast<s16x8*>(Xh + o) = hv;
      *keep_lo = lv;
      *keep_o = o;
    } else if constexpr (UPX == 2) {
      *reinterpret_cast<s16x8*>(Xh + o) = hv;
      if (PM != 2) *reinterpret_cast<s16x8*>(Xl + o) = lv;
    } else {
      *reinterpret_cast<s16x4*>(Xh + o) = s16x4{hv[0], hv[1], hv[2], hv[3]};
      if (PM != 2) *reinterpret_cast<s16x4*>(Xl + o) = s16x4{lv[0], lv[1], lv[2], lv[3]};
    }
  };
  UP up;
  float2 sx[XPIPE ? NLX : 1][4];
  auto load_d = [&](int t, int l) {
    const int f0 = (t / NRB) * FPT, y0 = (t % NRB) * RT;
    const int i = tid + l * 256;
    const int co = i / NPU, pt = DU * (i % NPU);
    const int fi = pt / (RT * W), y = (pt / W) % RT, xx = pt % W;
    const bool ok = i < NID && f0 + fi < F;
    // (a tile past the last one has f0 >= F: its lanes read frame 0)
    const int off = ok ? fi * (int)dy.fs + co * (int)HW + (y0 + y) * W + xx : 0;
    const float* q = dy.frame(f0 < F ? f0 : 0) + off;
    f32x4 v;
    if constexpr (DU == 4) v = *reinterpret_cast<const f32x4*>(q);
    else if constexpr (DU == 2) {
      const float2 u = *reinterpret_cast<const float2*>(q);
      v = f32x4{u.x, u.y, 0.f, 0.f};
    } else if constexpr (DU == 3) {
      v = f32x4{q[0], q[1], q[2], 0.f};
    } else {
      v = f32x4{*q, 0.f, 0.f, 0.f};
    }
    return ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
  };
  constexpr bool DPIPE = XPIPE || UPS || NLD * 4 <= 16;
  f32x4 sd[DPIPE ? NLD : 1];
  // PF: each dY unit's two windows: pooled gradients and code bytes
  constexpr int HPL = H / 2, WPL = W / 2;   // the pooled plane
  float2 pdp[PF ? NLD : 1];
  unsigned pcd[PF ? NLD : 1];
  auto load_pf = [&](int t, int l) {
    if constexpr (PF) {
      const int f0 = t / NRB, y0 = (t % NRB) * RT;
      const int i = tid + l * 256;
      const int co = i / NPU, pt = DU * (i % NPU);
      const int y = y0 + pt / W, xx = pt % W;
      const bool ok = i < NID && f0 < F;
      const int pw = (y >> 1) * WPL + (xx >> 1), c = co0 + co;
      const float* pp = ok ? pin.frame(f0) + (long long)c * (HPL * WPL) + pw : paig_zeros;
      pdp[l] = *reinterpret_cast<const float2*>(pp);
      const unsigned char* cb = ok ? pin.code + (long long)f0 * pin.code_fs + ((long long)(c >> 3) * (HPL * WPL) + pw) * 8 + (c & 7)
                                   : reinterpret_cast<const unsigned char*>(paig_zeros);
      pcd[l] = (unsigned)cb[0] | ((unsigned)cb[8] << 8);
    }
  };
  // dY unit l of tile t := ReLU'(y) * (dy + pooled gradient at the argmax)
  auto fold = [&](int t, int l, f32x4& v) {
    if constexpr (PF) {
      const int i = tid + l * 256;
      const int pr = ((((t % NRB) * RT) + (DU * (i % NPU)) / W) & 1) * 2;   // window row bits pr, pr + 1
#pragma unroll
      for (int w2 = 0; w2 < 2; ++w2) {
        const unsigned b = (pcd[l] >> (8 * w2)) & 255u;
        const int am = (int)(b >> 4) & 3;
        const float g = w2 ? pdp[l].y : pdp[l].x;
        const float vx = v[2 * w2] + (am == pr ? g : 0.f);
        const float vy = v[2 * w2 + 1] + (am == pr + 1 ? g : 0.f);
        v[2 * w2] = (b >> pr) & 1u ? vx : 0.f;
        v[2 * w2 + 1] = (b >> (pr + 1)) & 1u ? vy : 0.f;
      }
    }
  };
  auto issue = [&](int t) {
    if constexpr (UPS) {
      up.issue(x, F, (t / NRB) * FPT, (t % NRB) * RT, tid);
    } else if constexpr (XPIPE) {
#pragma unroll
      for (int l = 0; l < NLX; ++l) load_x(t, tid + l * 256, sx[l]);
    }
    if constexpr (DPIPE) {
#pragma unroll
      for (int l = 0; l < NLD; ++l) {
        sd[l] = load_d(t, l);
        load_pf(t, l);
      }
    }
  };
  // PF with prefetched dY: fold the tile before its max and staging
  auto fold_all = [&](int t) {
    if constexpr (PF && DPIPE) {
#pragma unroll
      for (int l = 0; l < NLD; ++l) fold(t, l, sd[l]);
    }
  };
  // PM 0 dY exponent.  dY held in registers before the barrier (prefetched)
  // publishes its tile max there (tile_max); synchronously loaded dY (DSYNC:
  // too many registers to prefetch) is staged with the running exponent and
  // checked after the barrier: a tile whose max would overflow f16 at that
  // scale (the block's first tile, or one > 2x any before) is staged again
  // with its own exponent.  One pass over the data in the steady state.
  constexpr bool DSYNC = !DPIPE;
  __shared__ float srd[4];
  auto rescale = [&](int nd) {   // block-uniform
    if (nd < ecd) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int j = 0; j < NTW; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[m][j][r] = __builtin_amdgcn_ldexpf(acc[m][j][r], nd - ecd);
    }
    ecd = nd;
    dsc = __builtin_amdgcn_ldexpf(1.f, ecd);
  };
  // dY staging of tile t (raw max into rd; bias partials on the first pass)
  auto stage_d = [&](int t, float& rd, bool first) {
#pragma unroll
    for (int l = 0; l < NLD; ++l) {
      const int i = tid + l * 256;
      if (NID % 256 != 0 && i >= NID) break;
      const int co = i / NPU, pt = DU * (i % NPU);
      f32x4 dv;
      if constexpr (DPIPE) {
        dv = sd[l];
      } else {
        dv = load_d(t, l);
        load_pf(t, l);
        fold(t, l, dv);
      }
      if (first) bacc[l] += (dv[0] + dv[1]) + (dv[2] + dv[3]);   // zeros past DU; unscaled
      s16x4 hv, lv;
      if constexpr (PM == 0) {
        if constexpr (DSYNC) rd = amax2(amax2(rd, dv[0], dv[1]), dv[2], dv[3]);
        const pf32x2 d0 = pf32x2{dv[0], dv[1]} * dsc, d1 = pf32x2{dv[2], dv[3]} * dsc;
        u32x2 a, b;
        { const HiLo q_ = split_pk(d0.x, d0.y); a[0] = q_.h; b[0] = q_.l; }
        { const HiLo q_ = split_pk(d1.x, d1.y); a[1] = q_.h; b[1] = q_.l; }
        hv = __builtin_bit_cast(s16x4, a);
        lv = __builtin_bit_cast(s16x4, b);
      } else {
        float dmx = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          short h, lo;
          split<PM>(dv[e], h, lo, dmx);
          hv[e] = h;
          lv[e] = lo;
        }
      }
      if constexpr (DU == 4) {
        *reinterpret_cast<s16x4*>(Dh + co * DP + pt) = hv;
        if (PM != 2) *reinterpret_cast<s16x4*>(Dl + co * DP + pt) = lv;
      } else {
#pragma unroll
        for (int e = 0; e < DU; ++e) {
          Dh[co * DP + pt + e] = hv[e];
          if (PM != 2) Dl[co * DP + pt + e] = lv[e];
        }
      }
    }
  };
  auto commit = [&](int t) {
    if constexpr (PM == 0 && !DSYNC && PAIG_SCALE_MODE < 2) {
      // this tile's dY exponent (block max published before the barrier); a
      // smaller one rescales the accumulators exactly
      const int td = f16_scale_exp(fmaxf(fmaxf(smax[0], smax[1]), fmaxf(smax[2], smax[3])));
      if (td < ecd) rescale(td);
    }
    float rd = 0.f;
    if constexpr (UPS) {
      const int f0 = (t / NRB) * FPT, y0 = (t % NRB) * RT;
      up.commit(Sl, tid);
      __syncthreads();
      if constexpr (C::SLA) {
        // the window lives in the lo X image's LDS: hi pieces now, lo pieces
        // held until every thread has read the window
        static_assert(W % 4 == 0 && UPX == 2, "SLA: 4-pixel items");
        constexpr int W4 = W / 4, NIT = ceil_div(NIX / 2, 256);
        s16x8 lk[NIT][2];
        int lo_o[NIT][2];
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
          const int i = tid + it * 256;
          lo_o[it][0] = -1;
          if ((NIX / 2) % 256 != 0 && i >= NIX / 2) break;
          const int q = i % W4, r = (i / W4) % ROWS, cq = (i / (W4 * ROWS)) % CQ, fi = i / (W4 * ROWS * CQ);
          const int gy = y0 + r - PADL;
          const bool ok = f0 + fi < F && gy >= 0 && gy < H;
          f32x4 o[4];
#pragma unroll
          for (int c = 0; c < 4; ++c)
            o[c] = (ok && cq * 4 + c < CINB) ? UP::row4(Sl, fi, cq * 4 + c, gy, y0, q) : f32x4{0.f, 0.f, 0.f, 0.f};
          const int ia = ((fi * CQ + cq) * ROWS + r) * W2 + 2 * q;
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            float2 v[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) v[c] = make_float2(o[c][2 * u], o[c][2 * u + 1]);
            put_x(ia + u, v, &lk[it][u], &lo_o[it][u]);
          }
        }
        __syncthreads();   // every read of the window is done
        // the lo image's halo columns (the window overwrote them)
        if (OFFX > 0) {
          for (int i = tid; i < FPT * ROWS * 2 * OFFX; i += 256) {
            const int hc = i % (2 * OFFX), r = i / (2 * OFFX);
            const int xc = hc < OFFX ? hc : W + hc;
            for (int cq = 0; cq < CQ; ++cq)
              *reinterpret_cast<s16x4*>(Xl + xplane(cq) + (r * TWPX + xc) * 4) = s16x4{0, 0, 0, 0};
          }
        }
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
          if (lo_o[it][0] < 0) break;
#pragma unroll
          for (int u = 0; u < 2; ++u) *reinterpret_cast<s16x8*>(Xl + lo_o[it][u]) = lk[it][u];
        }
      } else if constexpr (W % 4 == 0) {
        // units of 4 pixels x 4 channels (row4: shared taps and source reads)
        constexpr int W4 = W / 4;
#pragma unroll 1
        for (int i = tid; i < NIX / 2; i += 256) {
          const int q = i % W4, r = (i / W4) % ROWS, cq = (i / (W4 * ROWS)) % CQ, fi = i / (W4 * ROWS * CQ);
          const int gy = y0 + r - PADL;
          const bool ok = f0 + fi < F && gy >= 0 && gy < H;
          f32x4 o[4];
#pragma unroll
          for (int c = 0; c < 4; ++c)
            o[c] = (ok && cq * 4 + c < CINB) ? UP::row4(Sl, fi, cq * 4 + c, gy, y0, q) : f32x4{0.f, 0.f, 0.f, 0.f};
          const int ia = ((fi * CQ + cq) * ROWS + r) * W2 + 2 * q;
          float2 v[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) v[c] = make_float2(o[c][0], o[c][1]);
          put_x(ia, v);
#pragma unroll
          for (int c = 0; c < 4; ++c) v[c] = make_float2(o[c][2], o[c][3]);
          put_x(ia + 1, v);
        }
      } else {
#pragma unroll 1
        for (int i = tid; i < NIX; i += 256) {
          const int xp = UPX * (i % W2), r = (i / W2) % ROWS, cq = (i / (W2 * ROWS)) % CQ, fi = i / (W2 * ROWS * CQ);
          const int gy = y0 + r - PADL;
          const bool ok = f0 + fi < F && gy >= 0 && gy < H;
          float2 v[4];
#pragma unroll
          for (int c = 0; c < 4; ++c)
            v[c] = (ok && cq * 4 + c < CINB)
                       ? make_float2(UP::px1(Sl, fi, cq * 4 + c, gy, y0, xp),
                                     UPX == 2 ? UP::px1(Sl, fi, cq * 4 + c, gy, y0, xp + 1) : 0.f)
                       : make_float2(0.f, 0.f);
          put_x(i, v);
        }
      }
    } else if constexpr (XPIPE) {
#pragma unroll
      for (int l = 0; l < NLX; ++l) {
        const int i = tid + l * 256;
        if (NIX % 256 != 0 && i >= NIX) break;
        put_x(i, sx[l]);
      }
    } else {
#pragma unroll 1
      for (int i = tid; i < NIX; i += 256) {
        float2 v[4];
        load_x(t, i, v);
        put_x(i, v);
      }
    }
    stage_d(t, rd, true);
    if constexpr (PM == 0 && DSYNC) {
      rd = wave_max_u(rd);
      if (lane == 0) srd[wv] = rd;
    }
  };
  // after the post-commit barrier: re-stage synchronously loaded dY whose
  // tile max overflowed f16 at the running scale
  auto check_sync = [&](int t) {
    if constexpr (PM == 0 && DSYNC && PAIG_SCALE_MODE < 2) {
      const float md = uniform_f(fmaxf(fmaxf(srd[0], srd[1]), fmaxf(srd[2], srd[3])));
      if (md * dsc >= PAIG_F16_MAX) {   // block-uniform
        rescale(f16_scale_exp(md));
        float r1 = 0.f;
        stage_d(t, r1, false);
        __syncthreads();
      }
    }
  };

  // PM 0: this wave's max |dY| of the prefetched tile t into smax[wv] (read
  // by commit after the next barrier; the previous tile's reads finished
  // before the last one)
  auto tile_max = [&](int t) {
    if constexpr (!DSYNC) {
      float m = 0.f;
#pragma unroll
      for (int l = 0; l < NLD; ++l) m = amax2(amax2(m, sd[l][0], sd[l][1]), sd[l][2], sd[l][3]);
      m = wave_max_u(m);
      if (lane == 0) smax[wv] = m;
    }
  };

  if ((int)blockIdx.x < ntiles) issue(xcd_tile(blockIdx.x, ntiles));
  if (PM == 0 && xm.p) {
    // the launch's X exponent: max over the forward's per-block slots (their
    // loads overlap the first tile's)
    float m = 0.f;
    for (int i = tid * 4; i < xm.n; i += 1024) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(xm.p + i);
      m = fmaxf(m, fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])));
    }
    m = wave_max_u(m);
    if (lane == 0) smax[wv] = m;
    __syncthreads();
    m = fmaxf(fmaxf(smax[0], smax[1]), fmaxf(smax[2], smax[3]));
    if (m > 0.f) ecx = f16_scale_exp(m);   // all-zero slots (never written): the fixed scale, guarded
    __syncthreads();   // smax is reused by tile_max
  }
  xsc = __builtin_amdgcn_ldexpf(1.f, ecx);
  for (int lt = blockIdx.x; lt < ntiles; lt += gridDim.x) {
    const int tile = xcd_tile(lt, ntiles);
    fold_all(tile);
    if constexpr (PM == 0 && PAIG_SCALE_MODE < 2) tile_max(tile);
    __syncthreads();   // previous tile's fragment reads are done
    commit(tile);
    __syncthreads();
    check_sync(tile);
    // unconditional (branch-free for the load counting): past the last tile,
    // tile ntiles lies beyond frame F and every lane reads paig_zeros
    issue(lt + (int)gridDim.x < ntiles ? xcd_tile(lt + gridDim.x, ntiles) : ntiles);
#pragma unroll
    for (int kb = wp; kb < KB; kb += WP) {
      // k-block kb: 32 consecutive tile pixels, all in one frame
      const int p0 = kb * 32, fi = p0 / (RT * W), pr = p0 % (RT * W);
      const int base = (fi * ROWS + pr / W) * TWPX + pr % W;
      s16x8 ah[MT], al[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int co = m * 16 + (lane & 15);
        const int o = (co < COUTB ? co : co % COUTB) * DP + p0 + 8 * g;   // padded rows: finite, discarded
        ah[m] = *reinterpret_cast<const s16x8*>(Dh + o);
        al[m] = PM != 2 ? *reinterpret_cast<const s16x8*>(Dl + o) : ah[m];
      }
      int r0, r1;
      if constexpr (C::FAST) {
        r0 = (base + roff[0]) * 4;
        r1 = (base + roff[1]) * 4;
      } else {
        // pixel p of the k-block -> its image position (padded pixels: any
        // valid position; their dY is zero)
        auto posof = [&](int j) {
          int pp = p0 + j;
          if (pp >= TPXV) pp = 0;
          const int pf = pp / (RT * W), prr = pp % (RT * W);
          return ((pf * ROWS + prr / W) * TWPX + prr % W + (OFFX - PADL)) * 4;
        };
        r0 = posof(8 * g + qq);
        r1 = posof(8 * g + 4 + qq);
      }
      // B fragments one N-tile ahead: the transposed reads of tile jn+1 are
      // in flight during tile jn's MFMAs
      auto ldb = [&](int jn, s16x8& bh, s16x8& bl) {
        if (wn + jn * WN < NT) {   // wave-uniform: EXEC stays full for the tr reads
          bh = __builtin_shufflevector(tr_read(Xh + r0 + colt[jn]), tr_read(Xh + r1 + colt[jn]), 0, 1, 2, 3, 4, 5, 6,
                                       7);
          bl = PM != 2 ? __builtin_shufflevector(tr_read(Xl + r0 + colt[jn]), tr_read(Xl + r1 + colt[jn]), 0, 1, 2,
                                                 3, 4, 5, 6, 7)
                       : bh;
        }
      };
      s16x8 bh[2], bl[2];
      ldb(0, bh[0], bl[0]);
#pragma unroll
      for (int jn = 0; jn < NTW; ++jn) {
        if (jn + 1 < NTW) ldb(jn + 1, bh[(jn + 1) & 1], bl[(jn + 1) & 1]);
        if (wn + jn * WN < NT) {
#pragma unroll
          for (int m = 0; m < MT; ++m) acc[m][jn] = mma3<PM>(ah[m], al[m], bh[jn & 1], bl[jn & 1], acc[m][jn]);
        }
      }
    }
  }
  __syncthreads();
  // ---- cross-wave reduction (waves with equal wn, different wp) through LDS
  float* R = reinterpret_cast<float*>(lds16);   // [4 waves][MT][NTW][4][64]
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) R[(((wv * MT + m) * NTW + j) * 4 + r) * 64 + lane] = acc[m][j][r];
  __syncthreads();
  float* s = slab + (long long)blockIdx.x * C::SLAB;
  if (wp == 0) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        const int nt = wn + j * WN;
        if (nt >= NT) continue;
        const int col = nt * 16 + (lane & 15), cq = col >> 2;
        const int tap = cq / CQ, ci = (cq % CQ) * 4 + (col & 3);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = 0.f;
          for (int p = 0; p < WP; ++p) v += R[((((p * WN + wn) * MT + m) * NTW + j) * 4 + r) * 64 + lane];
          const int co = m * 16 + (lane >> 4) * 4 + r;
          if constexpr (PM == 0) v = __builtin_amdgcn_ldexpf(v, -(ecx + ecd));   // all waves share them
          if (co < COUTB && cq < NQ && ci < CINB) s[(co0 + co) * NCOL + (ci0 + ci) * KK + tap] = v;
        }
      }
  }
  // bias: every dY unit i (channel i / NPU) kept its fp32 partial in thread
  // i % 256, slot i / 256; one thread per channel sums them in unit order
  // (deterministic)
  __syncthreads();
  float* Rb = reinterpret_cast<float*>(lds16);   // [NLD][256]
#pragma unroll
  for (int l = 0; l < NLD; ++l) Rb[l * 256 + tid] = bacc[l];
  __syncthreads();
  if (tid < COUTB && blockIdx.y == 0) {   // bias: by the first input-channel slice
    float v = 0.f;
    for (int i = tid * NPU; i < (tid + 1) * NPU; ++i) v += Rb[(i / 256) * 256 + i % 256];
    s[COUT * NCOL + co0 + tid] = v;
  }
  if constexpr (PM == 0) f16_range_note(rmax);
}

// paig_debug_fwd_block_cap: at most this many persistent blocks per COUT
// slice in the split forward / dgrad launches (0: the resident count), so the
// ----------------------------------------------------------- weight prep
// The forward / dgrad kernels' weight images, built once per step for every
// conv: a header of one int per output channel (its weight exponent: the
// channel's max |w| scaled into [2^14, 2^15), so no magnitude overflows f16
// and every weight keeps 22 significant bits relative to its channel's
// largest), then the scaled weights split into f16 hi / lo, in fragment
// order over the whole COUT: entry (s, nt, lane) = 8 channels of k-chunk
// 4s + lane/16 for output channel 16 nt + lane%16; the lo image follows the
// hi one.  A block then stages its slice with coalesced 16-byte copies
// instead of one scattered 4-byte weight load (and split) per value, which
// measured 0.4-8 us per launch (the most on the small-frame, wide-channel
// layers).  The kernels' in-kernel staging (no image) forms the same
// exponents and values.
struct WPrepJob {
  const float* w;
  s16x8* out;
  int cin, cout, ks, dg;
};
constexpr int WPREP_MAX = 64;
struct WPrepJobs {
  WPrepJob j[WPREP_MAX];
  int blk0[WPREP_MAX + 1];   // first block of each job (one block per 16-channel N-tile)
  int n;
};
constexpr int WPREP_T = 256;

__device__ __forceinline__ int wprep_hdr_entries(int cout) { return (cout + 15) / 16 * 16 * 4 / 16; }

// one block per (job, N-tile of 16 output channels, WPREP_S k-steps): the
// 16 channel maxima (thread t: channel t % 16; every block of the tile forms
// them, from L2), their exponents, then its k-steps' entries.  8 k-steps:
// fewer blocks re-forming the same maxima (A/B over 2 / 4 / 8 / 16 / 64,
// tools/gpu_r6aq.sh, gpu_r6ar.sh: the first conv + prep launch 21.7-22.1 us
// for all of them, the step 98.1-98.5k seq/s at 8 vs 97.9-98.1k at 4)
#ifndef PAIG_WPREP_S
#define PAIG_WPREP_S 8
#endif
constexpr int WPREP_S = PAIG_WPREP_S;
__device__ __forceinline__ void conv_wprep_body(const WPrepJobs& jobs, int bid) {
  int q = 0;
  while (q + 1 < jobs.n && bid >= jobs.blk0[q + 1]) ++q;
  const WPrepJob jb = jobs.j[q];
  if (jb.dg == 2) {   // a dense layer's weight [cout][cin] -> out [cin][cout] fp32 (32 x 32 tiles)
    __shared__ float T[32][33];
    const int bl = bid - jobs.blk0[q], tx = (bl % ((jb.cin + 31) / 32)) * 32,
              ty = (bl / ((jb.cin + 31) / 32)) * 32, c = threadIdx.x & 31, r = threadIdx.x >> 5;
    for (int y = r; y < 32; y += WPREP_T / 32)
      if (ty + y < jb.cout && tx + c < jb.cin) T[y][c] = jb.w[(long long)(ty + y) * jb.cin + tx + c];
    __syncthreads();
    float* o = reinterpret_cast<float*>(jb.out);
    for (int y = r; y < 32; y += WPREP_T / 32)
      if (tx + y < jb.cin && ty + c < jb.cout) o[(long long)(tx + y) * jb.cout + ty + c] = T[c][y];
    return;
  }
  const int KK = jb.ks * jb.ks, CC = (jb.cin + 7) / 8, KC = KK * CC, NTT = (jb.cout + 15) / 16, NS = (KC + 3) / 4;
  const int NSC = (NS + WPREP_S - 1) / WPREP_S;   // k-step chunks per N-tile
  const int bl = bid - jobs.blk0[q], nt = bl / NSC, s0 = (bl % NSC) * WPREP_S;
  const int tid = threadIdx.x;
  auto wv = [&](int kc, int j, int co) {
    float v = 0.f;
    if (kc < KC && co < jb.cout) {
      const int tap = kc / CC, ci = (kc % CC) * 8 + j;
      if (ci < jb.cin) v = jb.dg ? jb.w[(ci * jb.cout + co) * KK + (KK - 1 - tap)] : jb.w[(co * jb.cin + ci) * KK + tap];
    }
    return v;
  };
  __shared__ float red[WPREP_T];
  __shared__ int ex[16];
  const int cl = tid & 15, co = nt * 16 + cl;
  // (unrolled: the loads of one thread are independent, keep 8 in flight)
  float m = 0.f;
#pragma unroll 8
  for (int i = tid >> 4; i < KC * 8; i += WPREP_T / 16) m = fmaxf(m, fabsf(wv(i >> 3, i & 7, co)));
  red[tid] = m;
  __syncthreads();
  if (tid < 16) {
    float mm = 0.f;
    for (int r = 0; r < WPREP_T / 16; ++r) mm = fmaxf(mm, red[r * 16 + tid]);
    ex[tid] = f16_scale_exp_v(mm);
    if (s0 == 0) reinterpret_cast<int*>(jb.out)[nt * 16 + tid] = ex[tid];
  }
  __syncthreads();
  const int HDR = wprep_hdr_entries(jb.cout), ENT = NS * NTT * 64;
  short* img = reinterpret_cast<short*>(jb.out + HDR);
  // this block's entries: (s, lane) -> value index t = ((s - s0) * 64 + lane) * 8 + j
  const int ns = NS - s0 < WPREP_S ? NS - s0 : WPREP_S;
#pragma unroll 8
  for (int t = tid; t < ns * 64 * 8; t += WPREP_T) {
    const int j = t & 7, ln = (t >> 3) & 63, s = s0 + (t >> 9);
    const int kc = 4 * s + (ln >> 4), c = nt * 16 + (ln & 15);
    float rm = 0.f;
    short h, l;
    split<0>(__builtin_amdgcn_ldexpf(wv(kc, j, c), ex[ln & 15]), h, l, rm);
    const long long e = (long long)(s * NTT + nt) * 64 + ln;
    img[e * 8 + j] = h;
    img[((long long)ENT + e) * 8 + j] = l;
  }
}

__global__ void __launch_bounds__(WPREP_T) conv_wprep_k(WPrepJobs jobs) { conv_wprep_body(jobs, blockIdx.x); }

// The step's weight prep and the U-Net's first forward conv (3 input
// channels) in one launch: blocks 0 .. nwp-1 run the prep jobs, the others
// the forward, which stages its own (tiny) weights in-kernel -- the same
// exponents and values as its image -- so nothing in the launch waits on the
// prep (paig_conv_wprep_defer)
template <int CIN, int COUT, int H, int W, int KS, int PM>
__global__ void __launch_bounds__(256, 2)
conv_fwd_wprep_k(FView in, FViewW out, FView aux, const float* __restrict__ w, const float* __restrict__ bias, int F,
                 int flags, int ntiles, XMax xm, PoolOut pout, WPrepJobs jobs, int nwp) {
  if ((int)blockIdx.x < nwp) {   // block-uniform
    conv_wprep_body(jobs, blockIdx.x);
    return;
  }
  conv_fwd_split_body<CIN, COUT, H, W, KS, false, false, PM>(in, out, aux, w, bias, F, flags, ntiles, xm, nullptr, pout,
                                                            (int)blockIdx.x - nwp, (int)gridDim.x - nwp);
}

// deferred weight prep (paig_conv_wprep_defer): taken by the next eligible
// split forward (above), launched on its own before any other one
WPrepJobs g_wpend{};
int g_wpend_blocks = 0;   // 0: none pending
int wprep_build(WPrepJobs& jobs, int n, const float* const* w, const int* cin, const int* cout, const int* ks,
                const int* dg, void* const* out, int* blocks_out) {
  jobs = WPrepJobs{};
  jobs.n = n;
  int blocks = 0;
  for (int q = 0; q < n; ++q) {
    PAIG_REQUIRE(w[q] && out[q] && cin[q] > 0 && cout[q] > 0 && ks[q] > 0, "conv_wprep: job %d", q);
    PAIG_REQUIRE(((uintptr_t)out[q] & 15) == 0, "conv_wprep: job %d output not 16-byte aligned", q);
    jobs.j[q] = WPrepJob{w[q], static_cast<s16x8*>(out[q]), cin[q], cout[q], ks[q], dg[q]};
    jobs.blk0[q] = blocks;
    if (dg[q] == 2) {   // dense transpose job
      blocks += (cin[q] + 31) / 32 * ((cout[q] + 31) / 32);
      continue;
    }
    const int NS = (ks[q] * ks[q] * ((cin[q] + 7) / 8) + 3) / 4;
    blocks += (cout[q] + 15) / 16 * ((NS + WPREP_S - 1) / WPREP_S);
  }
  jobs.blk0[n] = blocks;
  *blocks_out = blocks;
  return 0;
}
int wprep_flush(hipStream_t st) {
  if (!g_wpend_blocks) return 0;
  const int nb = g_wpend_blocks;
  g_wpend_blocks = 0;
  hipLaunchKernelGGL(conv_wprep_k, dim3(nb), dim3(WPREP_T), 0, st, g_wpend);
  PAIG_CHECK_LAUNCH();
  return 0;
}

// tests can make every block walk many tiles at small frame counts
static int g_fwd_block_cap = 0;
// pending pre-zero range for the next split forward (paig_conv_fwd_prezero)
static XMax g_prezero{};

template <int CIN, int COUT, int H, int W, int KS, bool DG, bool UPS, int PM, bool UPT = false, bool PF = false>
static int sfwd_launch(FView in, FViewW out, FView aux, const float* w, const float* b, int F, int flags,
                       hipStream_t st, XMax xm, const void* wp, PoolOut pout) {
  using C = SFwdCfg<CIN, COUT, H, W, KS, UPS, PM>;
  constexpr int LDS = C::LDS;
  static_assert(C::SLB == (UPS ? UpStage<CIN, H, W, C::FPT, C::RT>::SL * 4 : 0), "upsample window bytes");
  const int ntiles = cdiv(F, C::FPT) * (H / C::RT);
  // the fused-pool variant (its own instantiation: keeping the stored tile
  // live for the pool costs ~20 VGPRs, which the other launches must not pay)
  constexpr bool POOLABLE = C::POOLOK && !DG;
  auto k = PF ? conv_fwd_split_k<CIN, COUT, H, W, KS, DG, UPS, PM, false, false, PF>
         : UPT ? conv_fwd_split_k<CIN, COUT, H, W, KS, DG, UPS, PM, false, UPT>
              : (POOLABLE && (flags & 64)) ? conv_fwd_split_k<CIN, COUT, H, W, KS, DG, UPS, PM, POOLABLE>
                                           : conv_fwd_split_k<CIN, COUT, H, W, KS, DG, UPS, PM, false>;
  static int resident[2] = {0, 0};
  const int kv = (POOLABLE && (flags & 64)) ? 1 : 0;
  if (!resident[kv]) {
    if (LDS > 64 * 1024) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    resident[kv] = persistent_grid((const void*)k, LDS);
  }
  static const int bpc = [] {   // A/B: PAIG_FWD_BPC caps the forward's blocks per CU
    const char* e = getenv("PAIG_FWD_BPC");
    return e ? atoi(e) : 0;
  }();
  int res = resident[kv];
  if (bpc > 0 && res > bpc * 256) res = bpc * 256;
  int nb = res / C::NB;   // persistent blocks per COUT slice
  if (nb > (UPT ? F : ntiles)) nb = UPT ? F : ntiles;   // UPT: whole frames per block
  if (g_fwd_block_cap > 0 && nb > g_fwd_block_cap) nb = g_fwd_block_cap;   // tests: blocks walk many tiles
  if (nb < 1) nb = 1;
  if (PM != 0 || DG) xm.p = nullptr;
  PAIG_REQUIRE(!xm.p || nb <= xm.n, "conv split fwd: %d blocks need more than %d xmax slots", nb, xm.n);
  if (xm.p && g_prezero.z) {   // this launch zeroes the later layers' slots
    xm.z = g_prezero.z;
    xm.zn = g_prezero.zn;
    g_prezero = XMax{};
  }
  if (PF) PAIG_REQUIRE(pout.p && pout.code, "conv split dgrad: the pool fold needs the pooled gradient and codes");
  else if (flags & 64) PAIG_REQUIRE(C::POOLOK && pout.p, "conv split fwd: no fused pool for Cin=%d Cout=%d H=%d", CIN, COUT, H);
  if constexpr (CIN == 3 && PM == 0 && !DG && !UPS && !UPT && !PF && C::NB == 1) {
    if (g_wpend_blocks && !(flags & 64)) {   // the deferred weight prep rides in this launch
      auto km = conv_fwd_wprep_k<CIN, COUT, H, W, KS, PM>;
      static bool attr = false;
      if (!attr && LDS > 64 * 1024) (void)hipFuncSetAttribute((const void*)km, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
      attr = true;
      const int nwp = g_wpend_blocks;
      g_wpend_blocks = 0;
      hipLaunchKernelGGL(km, dim3(nwp + nb), dim3(256), LDS, st, in, out, aux, w, b, F, flags, ntiles, xm, pout, g_wpend,
                         nwp);
      PAIG_CHECK_LAUNCH();
      return 0;
    }
  }
  if (int rc = wprep_flush(st)) return rc;   // a forward that reads the images: they come first
  hipLaunchKernelGGL(k, dim3(nb, C::NB), dim3(256), LDS, st, in, out, aux, w, b, F, flags, ntiles, xm,
                     PM == 0 ? static_cast<const s16x8*>(wp) : nullptr, pout);
  PAIG_CHECK_LAUNCH();
  return 0;
}

template <int CIN, int COUT, int H, int W, int KS, bool UPS, int PM, bool PF = false>
static int swg_launch(FView x, FView dy, float* slab, int nblk_max, int* nblk_out, int F, hipStream_t st, XMax xm,
                      PoolOut pin = PoolOut{nullptr, 0, nullptr, 0}) {
  using C = SWgCfg<CIN, COUT, H, W, KS, UPS, PM>;
  constexpr int STG = C::STG + (UPS && !C::SLA ? UpStage<C::CINB, H, W, C::FPT, C::RT>::SL * 4 : 0);
  constexpr int LDS = STG > C::RED ? STG : C::RED;
  const int ntiles = cdiv(F, C::FPT) * (H / C::RT);
  auto k = conv_wgrad_split_k<CIN, COUT, H, W, KS, UPS, PM, PF>;
  if constexpr (PF) PAIG_REQUIRE(pin.p && pin.code, "conv split wgrad: the pool fold needs the pooled gradient and codes");
  static int resident = 0;
  if (!resident) {
    if (LDS > 64 * 1024) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    resident = persistent_grid((const void*)k, LDS);
  }
  // one wave of co-resident persistent blocks: more would leave a partial
  // second wave running at a fraction of the chip (and add slab rows)
  int nb = ntiles < nblk_max ? ntiles : nblk_max;
  if (nb > resident / (C::NSI * C::NSO)) nb = resident / (C::NSI * C::NSO);
  if (nb < 1) nb = 1;
  *nblk_out = nb;
  PAIG_REQUIRE(!xm.p || (xm.n % 4 == 0 && (reinterpret_cast<uintptr_t>(xm.p) & 15) == 0),
               "conv split wgrad: xmax needs 16-byte alignment and a multiple of 4 slots (%d)", xm.n);
  hipLaunchKernelGGL(k, dim3(nb, C::NSI, C::NSO), dim3(256), LDS, st, x, dy, slab, F, ntiles, xm, pin);
  PAIG_CHECK_LAUNCH();
  return 0;
}

// (CIN, COUT, H, KS) of the ShallowUNet(hidden 8) shapes at 32x32: forward
// and dgrad kernel shapes (dgrad shapes are (layer Cout, layer Cin)); *_UP:
// the convs whose input is the fused 2x upsample (c7, c10)
#define PAIG_SPLIT_FWD(X)                                                                                 \
  X(3, 8, 32, 3) X(8, 8, 32, 3) X(8, 16, 16, 3) X(16, 16, 16, 3) X(16, 32, 8, 3) X(32, 32, 8, 3)         \
  X(32, 16, 16, 3) X(16, 16, 32, 3) X(24, 8, 32, 3) X(8, 2, 32, 1) X(16, 8, 16, 3) X(8, 24, 32, 3)       \
  X(2, 8, 32, 1) X(32, 16, 8, 3) X(16, 32, 16, 3)                                                         \
  PAIG_SPLIT_FWD_3BP(X) PAIG_SPLIT_FWD_UNET(X)
#define PAIG_SPLIT_WG(X)                                                                                  \
  X(3, 8, 32, 3) X(8, 8, 32, 3) X(8, 16, 16, 3) X(16, 16, 16, 3) X(16, 32, 8, 3) X(32, 32, 8, 3)         \
  X(32, 16, 16, 3) X(16, 16, 32, 3) X(24, 8, 32, 3) X(8, 2, 32, 1)                                        \
  PAIG_SPLIT_WG_3BP(X) PAIG_SPLIT_WG_UNET(X)
#define PAIG_SPLIT_UP(X)                                                                                  \
  X(32, 16, 16, 3) X(16, 16, 32, 3) X(32, 16, 18, 3) X(16, 16, 36, 3) X(128, 32, 16, 3) X(64, 32, 32, 3) \
  X(32, 32, 64, 3)
// UNet convs whose output's max pool is folded into their separate weight
// gradient's dY staging and their data gradient's input staging (flags & 64;
// c4: too wide for the fused layer backward): (Cin, Cout) of the layer.  c6
// (64 -> 64 @ 16^2) keeps the standalone pool backward: its folding dgrad
// spills 32 VGPRs (the plain one already takes 240)
#define PAIG_SPLIT_PF(X) X(32, 32, 32, 3) PAIG_SPLIT_PF_C6(X)
#ifndef PAIG_PF_C6
#define PAIG_PF_C6 0   // A/B builds: 1 = c6 (64 -> 64 @ 16^2) folds pool3 too (its dgrad spills 32 VGPRs)
#endif
#if PAIG_PF_C6
#define PAIG_SPLIT_PF_C6(X) X(64, 64, 16, 3)
#else
#define PAIG_SPLIT_PF_C6(X)
#endif
// dgrad shapes (layer Cout, layer Cin) of the UNet convs whose input is the
// 2x upsample (c9, c12, c15) with the transposed-upsample epilogue (UPT)
#define PAIG_SPLIT_UPT(X) X(32, 128, 16, 3) X(32, 64, 32, 3) X(32, 32, 64, 3)
// 3bp_color (ShallowUNet hidden 8 on 36 x 36 frames, K = 3 objects): levels
// 36 / 18 / 9; tiles of 6 rows (36), 9 rows (18) or 3 frames (9 x 9)
#define PAIG_SPLIT_FWD_3BP(X)                                                                             \
  X(3, 8, 36, 3) X(8, 8, 36, 3) X(8, 16, 18, 3) X(16, 16, 18, 3) X(16, 32, 9, 3) X(32, 32, 9, 3)         \
  X(32, 16, 18, 3) X(16, 16, 36, 3) X(24, 8, 36, 3) X(8, 3, 36, 1) X(16, 8, 18, 3) X(32, 16, 9, 3)       \
  X(16, 32, 18, 3) X(8, 24, 36, 3) X(3, 8, 36, 1)
// mnist_spring_color (UNet hidden 16 on 64 x 64 frames): levels 64 / 32 /
// 16 / 8, 3..128 channels; forward then dgrad-only shapes
#define PAIG_SPLIT_FWD_UNET(X)                                                                            \
  X(3, 16, 64, 3) X(16, 16, 64, 3) X(16, 32, 32, 3) X(32, 32, 32, 3) X(32, 64, 16, 3) X(64, 64, 16, 3)   \
  X(64, 128, 8, 3) X(128, 128, 8, 3) X(96, 64, 16, 3) X(64, 32, 32, 3) X(48, 16, 64, 3) X(16, 2, 64, 1)   \
  X(32, 16, 32, 3) X(64, 32, 16, 3) X(128, 64, 8, 3) X(32, 128, 16, 3) X(64, 96, 16, 3) X(32, 64, 32, 3)  \
  X(32, 32, 64, 3) X(16, 48, 64, 3) X(2, 16, 64, 1)
#define PAIG_SPLIT_WG_UNET(X)                                                                             \
  X(3, 16, 64, 3) X(16, 16, 64, 3) X(16, 32, 32, 3) X(32, 32, 32, 3) X(32, 64, 16, 3) X(64, 64, 16, 3)   \
  X(64, 128, 8, 3) X(128, 128, 8, 3) X(96, 64, 16, 3) X(64, 32, 32, 3) X(48, 16, 64, 3) X(16, 2, 64, 1)
#define PAIG_SPLIT_WG_3BP(X)                                                                              \
  X(3, 8, 36, 3) X(8, 8, 36, 3) X(8, 16, 18, 3) X(16, 16, 18, 3) X(16, 32, 9, 3) X(32, 32, 9, 3)         \
  X(32, 16, 18, 3) X(16, 16, 36, 3) X(24, 8, 36, 3) X(8, 3, 36, 1)

}  // namespace

// flags & 128: split precision (f16 x3 forward and scaled dgrad), flags & 256:
// bf16 hi only.  Returns 1 if the shape is instantiated here (rc in *rc).
int paig_conv_split_fwd(FView in, FViewW out, FView aux, const float* w, const float* b, int F, int Cin, int Cout,
                        int H, int W, int ks, int flags, hipStream_t st, int* rc, XMax xm, const void* wp,
                        PoolOut pout) {
  const bool dg = (flags & 8) != 0, up = (flags & 32) != 0, b16 = (flags & 256) != 0;
  const int fl = flags & (7 | 64);
  if (H != W || !(flags & (128 | 256))) return 0;
  if (in.grp > 0 && H * W < 256) return 0;   // multi-frame tiles step frames by a plain stride
  if (dg && (flags & 64)) {   // dgrad with the output max pool's backward folded into its input staging (PF)
    if (up || b16 || (flags & 512)) return 0;
#define PAIG_CASE(CI, CO, HH, K)                                                                          \
    if (Cin == CO && Cout == CI && H == HH && ks == K) {                                                  \
      *rc = sfwd_launch<CO, CI, HH, HH, K, true, false, 0, false, true>(in, out, aux, w, b, F, fl & 7, st, xm, wp, pout); \
      return 1;                                                                                           \
    }
    PAIG_SPLIT_PF(PAIG_CASE)
#undef PAIG_CASE
    return 0;
  }
  if (flags & 512) {   // dgrad writing the transposed upsample of dX (UPT)
    if (!dg || up || b16 || (flags & (4 | 64))) return 0;
#define PAIG_CASE(CI, CO, HH, K)                                                                          \
    if (Cin == CI && Cout == CO && H == HH && ks == K) {                                                  \
      *rc = sfwd_launch<CI, CO, HH, HH, K, true, false, 0, true>(in, out, aux, w, b, F, fl, st, xm, wp, pout); \
      return 1;                                                                                           \
    }
    PAIG_SPLIT_UPT(PAIG_CASE)
#undef PAIG_CASE
    return 0;
  }
  if (up) {
    if (dg) return 0;
#define PAIG_CASE(CI, CO, HH, K)                                                                          \
    if (Cin == CI && Cout == CO && H == HH && ks == K) {                                                  \
      *rc = b16 ? sfwd_launch<CI, CO, HH, HH, K, false, true, 2>(in, out, aux, w, b, F, fl, st, xm, wp, pout)           \
                : sfwd_launch<CI, CO, HH, HH, K, false, true, 0>(in, out, aux, w, b, F, fl, st, xm, wp, pout);          \
      return 1;                                                                                           \
    }
    PAIG_SPLIT_UP(PAIG_CASE)
#undef PAIG_CASE
    return 0;
  }
#define PAIG_CASE(CI, CO, HH, K)                                                                            \
  if (Cin == CI && Cout == CO && H == HH && ks == K) {                                                      \
    if (b16)                                                                                                \
      *rc = dg ? sfwd_launch<CI, CO, HH, HH, K, true, false, 2>(in, out, aux, w, b, F, fl, st, xm, wp, pout)              \
               : sfwd_launch<CI, CO, HH, HH, K, false, false, 2>(in, out, aux, w, b, F, fl, st, xm, wp, pout);            \
    else                                                                                                    \
      *rc = dg ? sfwd_launch<CI, CO, HH, HH, K, true, false, 0>(in, out, aux, w, b, F, fl, st, xm, wp, pout)              \
               : sfwd_launch<CI, CO, HH, HH, K, false, false, 0>(in, out, aux, w, b, F, fl, st, xm, wp, pout);            \
    return 1;                                                                                               \
  }
  PAIG_SPLIT_FWD(PAIG_CASE)
#undef PAIG_CASE
  return 0;
}

int paig_conv_split_wgrad(FView x, FView dy, float* slab, int nblk_max, int* nblk_out, int F, int Cin, int Cout,
                          int H, int W, int ks, int flags, hipStream_t st, int* rc, XMax xm, PoolOut pin) {
  const bool up = (flags & 32) != 0, b16 = (flags & 256) != 0;
  if (H != W || !(flags & (128 | 256))) return 0;
  if (x.grp > 0 && H * W < 256) return 0;   // multi-frame tiles step frames by a plain stride
  if (flags & 64) {   // the 2x2 max pool of the layer's output folded into the dY staging
    if (up || b16) return 0;
#define PAIG_CASE(CI, CO, HH, K)                                                                          \
    if (Cin == CI && Cout == CO && H == HH && ks == K) {                                                  \
      *rc = swg_launch<CI, CO, HH, HH, K, false, 0, true>(x, dy, slab, nblk_max, nblk_out, F, st, xm, pin);  \
      return 1;                                                                                           \
    }
    PAIG_SPLIT_PF(PAIG_CASE)
#undef PAIG_CASE
    return 0;
  }
  if (up) {
#define PAIG_CASE(CI, CO, HH, K)                                                                          \
    if (Cin == CI && Cout == CO && H == HH && ks == K) {                                                  \
      *rc = b16 ? swg_launch<CI, CO, HH, HH, K, true, 2>(x, dy, slab, nblk_max, nblk_out, F, st, xm)          \
                : swg_launch<CI, CO, HH, HH, K, true, 0>(x, dy, slab, nblk_max, nblk_out, F, st, xm);         \
      return 1;                                                                                           \
    }
    PAIG_SPLIT_UP(PAIG_CASE)
#undef PAIG_CASE
    return 0;
  }
#define PAIG_CASE(CI, CO, HH, K)                                                                          \
  if (Cin == CI && Cout == CO && H == HH && ks == K) {                                                    \
    *rc = b16 ? swg_launch<CI, CO, HH, HH, K, false, 2>(x, dy, slab, nblk_max, nblk_out, F, st, xm)           \
              : swg_launch<CI, CO, HH, HH, K, false, 0>(x, dy, slab, nblk_max, nblk_out, F, st, xm);          \
    return 1;                                                                                             \
  }
  PAIG_SPLIT_WG(PAIG_CASE)
#undef PAIG_CASE
  return 0;
}

// 1 if paig_conv_split_fwd (what 0) / paig_conv_split_wgrad (what 1) has the shape
int paig_conv_split_supported(int what, int Cin, int Cout, int H, int W, int ks, int flags) {
  if (H != W) return 0;
  const bool up = (flags & 32) != 0, dg = (flags & 8) != 0;
  if ((flags & 64) && (what == 1 || dg)) {   // the output max pool's backward folded (wgrad / dgrad staging)
    if (up || !(flags & 128) || (flags & (256 | 512))) return 0;
#define PAIG_CASE(CI, CO, HH, K)                                                                         \
    if (what == 1 ? (Cin == CI && Cout == CO) : (Cin == CO && Cout == CI)) {                             \
      if (H == HH && ks == K) return 1;                                                                  \
    }
    PAIG_SPLIT_PF(PAIG_CASE)
#undef PAIG_CASE
    return 0;
  }
  if (flags & 64) {   // forward with the fused 2x2 max pool of its output
    if (what != 0 || up || dg || !(flags & (128 | 256))) return 0;
    const bool b16 = (flags & 256) != 0;
#define PAIG_CASE(CI, CO, HH, K)                                                                         \
    if (Cin == CI && Cout == CO && H == HH && ks == K)                                                   \
      return b16 ? SFwdCfg<CI, CO, HH, HH, K, false, 2>::POOLOK : SFwdCfg<CI, CO, HH, HH, K, false, 0>::POOLOK;
    PAIG_SPLIT_FWD(PAIG_CASE)
#undef PAIG_CASE
    return 0;
  }
#define PAIG_CASE(CI, CO, HH, K) \
  if (Cin == CI && Cout == CO && H == HH && ks == K) return 1;
  if (flags & 512) {
    if (what != 0 || !dg || up || (flags & (4 | 64 | 256)) || !(flags & 128)) return 0;
    PAIG_SPLIT_UPT(PAIG_CASE)
    return 0;
  }
  if (up) {
    if (dg) return 0;
    PAIG_SPLIT_UP(PAIG_CASE)
    return 0;
  }
  if (what == 0) {
    PAIG_SPLIT_FWD(PAIG_CASE)
  } else {
    PAIG_SPLIT_WG(PAIG_CASE)
  }
#undef PAIG_CASE
  return 0;
}

void paig_conv_fwd_prezero(float* z, int zn) {
  g_prezero.z = z;
  g_prezero.zn = zn;
}
bool paig_conv_fwd_prezero_pending() {
  const bool pend = g_prezero.z != nullptr;
  g_prezero = XMax{};
  return pend;
}

extern "C" {

int paig_debug_fwd_block_cap(int cap) {
  const int prev = g_fwd_block_cap;
  g_fwd_block_cap = cap > 0 ? cap : 0;
  return prev;
}

// 16-bit elements of one prepped weight image (channel-exponent header + hi
// + lo) for a forward / dgrad kernel with cin input and cout output channels
long long paig_conv_wprep_size(int cin, int cout, int ks) {
  const int KC = ks * ks * ((cin + 7) / 8), NS = (KC + 3) / 4, NTT = (cout + 15) / 16;
  return 2ll * NS * NTT * 64 * 8 + (long long)NTT * 16 * 2;
}

int paig_conv_wprep(int n, const float* const* w, const int* cin, const int* cout, const int* ks, const int* dg,
                    void* const* out, void* stream) {
  if (int rc = wprep_flush((hipStream_t)stream)) return rc;   // (in stream order)
  for (int b = 0; b < n; b += WPREP_MAX) {
    WPrepJobs jobs;
    int blocks = 0;
    const int m = n - b < WPREP_MAX ? n - b : WPREP_MAX;
    if (int rc = wprep_build(jobs, m, w + b, cin + b, cout + b, ks + b, dg + b, out + b, &blocks)) return rc;
    hipLaunchKernelGGL(conv_wprep_k, dim3(blocks), dim3(WPREP_T), 0, (hipStream_t)stream, jobs);
    PAIG_CHECK_LAUNCH();
  }
  return 0;
}

// paig_conv_wprep deferred to the next split forward launch on this thread:
// the U-Net's first layer (3 input channels, split arithmetic) runs the jobs
// in extra blocks of its own launch; any other split forward launches them
// first, and paig_unet_fwd_ex flushes them before it returns.  More than one
// launch's worth of jobs, or jobs still pending: launched now.
int paig_conv_wprep_defer(int n, const float* const* w, const int* cin, const int* cout, const int* ks, const int* dg,
                          void* const* out, void* stream) {
  if (n > WPREP_MAX || g_wpend_blocks) return paig_conv_wprep(n, w, cin, cout, ks, dg, out, stream);
  if (n <= 0) return 0;
  int blocks = 0;
  if (int rc = wprep_build(g_wpend, n, w, cin, cout, ks, dg, out, &blocks)) return rc;
  g_wpend_blocks = blocks;
  return 0;
}

int paig_conv_wprep_flush(void* stream) { return wprep_flush((hipStream_t)stream); }

}  // extern "C"

PAIG_F16_RANGE_ACCESSOR(paig_f16_range_conv)
