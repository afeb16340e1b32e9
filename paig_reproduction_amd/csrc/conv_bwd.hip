// Fused backward of one U-Net convolution layer on the gfx950 16-bit matrix
// cores (split-precision operands, conv_split.hip's arithmetic).  Reference:
// aten convolution_backward behind nn/network/blocks.py:246-276 (ShallowUNet)
// and :113-170 (UNet); one launch replaces the layer's data-gradient and
// weight-gradient kernels (paig_conv2d_fwd_pw flags & 8, paig_conv2d_wgrad_ex).
//
// Per persistent tile (whole rows of one frame, or whole frames; <= 256
// pixels) the block stages ONCE
//   * dY with a one-pixel halo as an NHWC 16-bit image (8 channels = one
//     16-byte slot per pixel, odd pixel pitch): the data gradient's A operand
//     (one ds_read_b128 per fragment, as the dgrad kernel reads it) AND, read
//     with ds_read_b64_tr_b16 (4 pixels x 16 channels -> 4 pixels of one
//     channel per lane), the weight gradient's A operand dY[co][pixel];
//   * X with a one-pixel halo as 4-channel quad planes (the weight gradient's
//     B operand, transposed reads whose per-lane row address absorbs the tap
//     shift, as conv_wgrad_split_k);
// and computes
//   * dX[pixel][ci] = sum_(tap, co) dY[pixel + tap][co] * W[co][ci][flip(tap)]
//     for the tile's pixels (ReLU' of the layer input and accumulation into
//     the existing gradient in the epilogue, as the dgrad kernel);
//   * dW[co][ci][tap] += sum_pixel dY[co][pixel] * X[pixel + tap][ci] and
//     db[co] += sum_pixel dY[co][pixel] (exact fp32, from the staging
//     registers), one slab row per block (the same slab layout as the wgrad
//     kernel: one batched deterministic reduction afterwards).
// What the two separate kernels did twice is done once: dY read from HBM and
// converted to 16-bit pieces once (the dgrad and the wgrad each did), X read
// once (the wgrad's staging and the dgrad's ReLU' mask read it separately).
//
// Scales (PM 0, f16 hi/lo): X by one power of two per launch (the forward's
// recorded maximum, xmax); dY by one power of two per tile (its own max; the
// weight-gradient accumulators follow each tile's exponent by exact power-of-
// two rescaling); weights per output channel (paig_conv_wprep's header).  The
// data gradient of a tile is complete in the tile, so its epilogue takes the
// exponents back out exactly.  PM 2: bf16 hi only, unscaled (BASELINE config
// #2).
#include "split_common.h"

#include <stdlib.h>

#ifndef PAIG_BWD_MINW
#define PAIG_BWD_MINW 0   // A/B builds: force the blocks per CU the kernels are compiled for
#endif
#ifndef PAIG_BWD_UPS2
#define PAIG_BWD_UPS2 1   // A/B builds: 0 = one-row upsample staging items
#endif
#ifndef PAIG_BWD_TPX_C10
#define PAIG_BWD_TPX_C10 0   // A/B builds: tile pixels / blocks per CU of c10 (16 -> 16 @ 32, upsample fold)
#define PAIG_BWD_MINW_C10 0
#endif
#ifndef PAIG_BWD_PSD_EVEN_C10
#define PAIG_BWD_PSD_EVEN_C10 0   // A/B builds: c10's dY image at an even pixel pitch (less LDS, more conflicts)
#endif
#ifndef PAIG_BWD_AUXP
#define PAIG_BWD_AUXP 1   // A/B builds: 0 = the epilogue loads its ReLU' mask when it needs it
#endif

// Diagnostic build only (-DPAIG_BWD_STAMPS, tools/bwd_bench.py): per wave,
// s_memtime cycle sums of the tile loop's phases (0 setup, 1 prefetch wait +
// max + barrier, 2 commit, 3 issue, 4 weight gradient, 5 data gradient, 6
// epilogue, 7 slab write; inside the commit: 8 dY staging, 9 UPS window +
// halo, 10 its barrier, 11 the upsampled X staging) and the tile count, stored
// by lane 0 (vector stores)
#ifdef PAIG_BWD_STAMPS
__device__ unsigned long long paig_bwd_stamps[4096][4][13];
#define PAIG_BSTAMP(k)                                      \
  do {                                                      \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    st_acc[k] += t_ - st_last;                              \
    st_last = t_;                                           \
  } while (0)
#else
#define PAIG_BSTAMP(k) \
  do {                 \
  } while (0)
#endif

namespace {

// LDS bytes of a block at tiles of <= tpx pixels (both images, the weights,
// the fused-upsample window)
constexpr int sbwd_lds(int CIN, int COUT, int H, int W, bool UPS, int PM, int tpx) {
  const int FPT = H * W <= tpx ? tpx / (H * W) : 1, RT = H * W <= tpx ? H : rows_fit(H, W, tpx);
  const bool pe = PAIG_BWD_PSD_EVEN_C10 && UPS && CIN == 16 && COUT == 16 && H == 32;
  const int ROWS = RT + 2, ROWSD = ROWS + (UPS ? 2 : 0), CCD = rup(COUT, 8) / 8,
            PSD = CCD % 2 == 0 && !pe ? CCD + 1 : CCD;
  const int RPD = W == 8 ? to_mod16((W + 2) * PSD, 8) : (W + 2) * PSD;
  const int IMGD = (FPT * ROWSD * RPD + 2) * 8, WIMG = ceil_div(9 * CCD, 4) * ceil_div(CIN, 16) * 64 * 8;
  const int XIMG = rup(CIN, 4) / 4 * rup(FPT * ROWS * (W + 4) * 4 + 80, 128) * 2 * (PM == 2 ? 1 : 2);
  const int UPB = UPS ? CIN * (rup(FPT * (RT + 2) * W, 64) + 4) * 4 : 0;
  const int XREG = XIMG > UPB ? XIMG : UPB;
  return (IMGD + WIMG) * 2 * (PM == 2 ? 1 : 2) + XREG + (UPS ? up_window_floats(CIN, FPT, RT, W) * 4 : 0);
}
// pixels per tile: the largest of 256 / 128 / 64 whose staging lets two
// blocks share a CU (the 8 x 8 / 9 x 9 levels' multi-frame tiles and the
// 32-channel weight images would not)
constexpr int sbwd_tpx(int CIN, int COUT, int H, int W, bool UPS, int PM) {
  if (PAIG_BWD_TPX_C10 && UPS && CIN == 16 && COUT == 16 && H == 32) return PAIG_BWD_TPX_C10;
  for (int pass = 0; pass < 2; ++pass)
    for (int t = 256; t >= 64; t /= 2) {
      const int rt = H * W <= t ? H : rows_fit(H, W, t);
      if (UPS && (rt % 2 != 0 || H * W < t)) continue;   // the upsample fold: whole even row blocks of one frame
      if (sbwd_lds(CIN, COUT, H, W, UPS, PM, t) <= (pass == 0 ? LDS_MAX / 2 : LDS_MAX)) return t;
    }
  return 64;
}

// waves per SIMD (= blocks per CU) each shape compiles for without spilling
// (measured: -Rpass-analysis=kernel-resource-usage at 2 / 3 / 4)
constexpr int sbwd_minw(int CIN, int COUT, int H, int PM, bool PF) {
  if (PAIG_BWD_MINW_C10 && CIN == 16 && COUT == 16 && H == 32) return PAIG_BWD_MINW_C10;
  if (CIN == 8 && COUT == 8 && H == 32) return PF || PAIG_BWD_AUXP == 2 ? 3 : 4;
  if (PM == 2 && CIN == 8 && COUT == 16 && H == 16) return 3;
  if (PM == 2 && CIN == 24 && COUT == 8 && H == 32) return 3;
  if (CIN == 8 && COUT == 8 && H == 36) return PF ? 2 : 3;
  if (CIN == 8 && COUT == 16 && H == 18) return PM == 2 ? 4 : 3;
  if (CIN == 16 && COUT == 16 && H == 18) return PF ? 2 : 3;
  return 2;
}

// the shapes whose ReLU'-mask prefetch (AUXP) would spill registers at their
// blocks per CU (-Rpass-analysis=kernel-resource-usage); PAIG_BWD_AUXP=2
// (A/B builds) prefetches everywhere, c12's 8 -> 8 at three blocks per CU
constexpr bool sbwd_auxp(int CIN, int COUT, int H, int PM, bool UPS, bool PF) {
  if (PAIG_BWD_AUXP == 2) return true;
  if (CIN == 8 && COUT == 8 && (H == 32 || H == 36) && !PF) return false;
  if (CIN == 24 && COUT == 8 && (H == 36 || PM == 2)) return false;
  if (UPS && H == 36) return false;
  if (PM == 0) return !(PF && CIN == 16 && COUT == 16 && H == 16);
  return !((UPS && CIN == 32 && H == 16) || (CIN == 8 && COUT == 16 && H == 16));
}

// 4 waves split the weight-gradient N-tiles (each wave owns every 4th one
// over all pixels: no cross-wave reduction); the data gradient's M-tiles of
// 16 pixels are split over the waves as in the dgrad kernel
template <int CIN, int COUT, int H, int W, int KS, bool UPS, int PM, bool PF = false>
struct SBwdCfg {
  static constexpr int KK = KS * KS, PADL = KS / 2;
  static constexpr int NIMG = PM == 2 ? 1 : 2;
  static constexpr int TPX = sbwd_tpx(CIN, COUT, H, W, UPS, PM);
  static constexpr int FPT = H * W <= TPX ? TPX / (H * W) : 1;
  static constexpr int RT = H * W <= TPX ? H : rows_fit(H, W, TPX);
  static constexpr int TPXV = FPT * RT * W;                   // valid pixels per tile
  static constexpr int ROWS = RT + KS - 1;                    // X image rows (halo PADL)
  // fused upsample input (c7 / c10): the data gradient is formed for one
  // more row above and below the tile (EXT), so that the 2x upsample's
  // transpose of the tile's rows (low-resolution rows y0/2 .. (y0+RT)/2 - 1,
  // each fed by 4 full-resolution rows) completes inside the tile
  static constexpr int EXT = UPS ? 1 : 0;
  static constexpr int RTD = RT + 2 * EXT, ROWSD = ROWS + 2 * EXT;   // dX rows, dY image rows
  static constexpr int TPXD = FPT * RTD * W;                  // data-gradient pixels per tile
  // ---- dY image: NHWC, 8-channel slots, halo PADL
  static constexpr int CCD = rup(COUT, 8) / 8;
  static constexpr bool PSDE = PAIG_BWD_PSD_EVEN_C10 && UPS && CIN == 16 && COUT == 16 && H == 32;
  static constexpr int PSD = CCD % 2 == 0 && !PSDE ? CCD + 1 : CCD;   // odd pitch: 16 pixels -> 16 bank groups
  static constexpr int TWPX = W + 2 * PADL;
  static constexpr int RPD = W == 8 ? to_mod16(TWPX * PSD, 8) : TWPX * PSD;
  static constexpr int ZSLOT = FPT * ROWSD * RPD;             // a zero slot after the image
  static constexpr int IMGD = (ZSLOT + 2) * 8;                // (+1 spare slot: wgrad reads of 8-channel dY)
  // ---- data gradient: k = (tap, 8-channel chunk of dY), 4 chunks per MFMA k-step
  static constexpr int KC = KK * CCD, NS = ceil_div(KC, 4);
  static constexpr int NTD = ceil_div(CIN, 16);               // 16-channel tiles of dX
  static constexpr int NMT = ceil_div(TPXD, 16), MW = ceil_div(NMT, 4);
  static constexpr int WIMG = NS * NTD * 64 * 8;
  // ---- X image (weight gradient B operand): 4-channel quad planes
  static constexpr int CQ = rup(CIN, 4) / 4, NQ = KK * CQ, NTX = ceil_div(NQ, 4);
  static constexpr int OFFX = PADL > 0 ? 2 : 0, TWX = W + 2 * OFFX;
  static constexpr int XPL = rup(FPT * ROWS * TWX * 4 + 80, 128);
  static constexpr int XIMG = CQ * XPL;
  // ---- weight gradient: D[co][(tap, ci)], K = pixels in k-blocks of 32
  static constexpr int MT = ceil_div(COUT, 16), NTW = ceil_div(NTX, 4);
  // balanced N-tiles: NTF whole N-tiles per wave (wv + 4 j); the NTR = NTX % 4
  // tail N-tiles are split by k-blocks (wave wv takes kb % 4 == wv) instead of
  // going whole to waves 0 .. NTR-1, whose extra MFMAs every barrier waited
  // for (c12: 2 : 1 N-tiles); the tail partials are summed over the 4 waves
  // in LDS at the end, in wave order.  Not where the extra accumulators
  // spill (bf16 images; 3bp's 36-wide non-fused layers): whole tail N-tiles
  // to waves 0 .. NTR-1 there, as before
  static constexpr bool BAL = !(PM == 2 && (CIN == 24 || (UPS && CIN == 32) || H == 36 || H == 18)) && !(H == 36 && !UPS && !PF);
  static constexpr int NTF = BAL ? NTX / 4 : ceil_div(NTX, 4), NTR = BAL ? NTX % 4 : 0;
  static constexpr int KB = ceil_div(TPXV, 32);
  static constexpr int NCOL = CIN * KK, SLAB = COUT * NCOL + COUT;
  // ---- staging units: UPX pixels x (8 dY | 4 X) channels, pixel fastest
  static constexpr int UPX = W % 2 == 0 ? 2 : 1, W2 = W / UPX;
  static constexpr int NID = FPT * ROWSD * W2 * CCD, NLD = ceil_div(NID, 256);
  static constexpr int NIX = FPT * ROWS * W2 * CQ, NLX = ceil_div(NIX, 256);
  static constexpr int UPW = up_window_floats(CIN, FPT, RT, W);   // fused-upsample window (floats)
  // the X image's region (UPS: it later holds the tile's full-resolution dX)
  static constexpr int UPB = UPS ? CIN * (rup(FPT * (RT + 2) * W, 64) + 4) * 4 : 0;   // the dX tile's bytes
  static constexpr int XREG = XIMG * 2 * NIMG > UPB ? XIMG * 2 * NIMG : UPB;
  static constexpr int LDS = (IMGD + WIMG) * 2 * NIMG + XREG + (UPS ? UPW * 4 : 0);
  static constexpr bool VEC4 = W % 4 == 0;
  // X prefetched a tile ahead where its registers are cheap (else loaded
  // when staged)
  static constexpr bool XPIPE = !UPS && NLX * 8 <= 32;
  // blocks per CU the kernel is compiled for (__launch_bounds__): the most
  // that compile without register spills (sbwd_minw), within the LDS
  static constexpr int LDSB = LDS_MAX / (LDS > (NLD * 256 * 8 + 256) * 4 ? LDS : (NLD * 256 * 8 + 256) * 4);
  static constexpr int MW0 = PAIG_BWD_MINW > 0 ? PAIG_BWD_MINW : sbwd_minw(CIN, COUT, H, PM, PF);
  static constexpr int MINW = MW0 < LDSB ? MW0 : LDSB;
  static_assert(H % RT == 0, "RT divides H");
  static_assert(KS == 3, "3x3 layers (the 1x1 heads are fused elsewhere)");
  static_assert(!UPS || (FPT == 1 && RT % 2 == 0 && W % 2 == 0), "fused upsample: whole even row blocks of one frame");
  // PF: the 2x2 max pool of this layer's output folded into the dY staging
  // (a staging unit's pixel pair is one pooling window's columns)
  static_assert(!PF || (!UPS && UPX == 2 && COUT % 8 == 0 && H % 2 == 0), "pool fold: even widths, 8-channel chunks");
  // UPS: the tile's full-resolution dX rows [RTD][W] per channel (fp32) are
  // parked in the X image's region (free once the weight-gradient MFMAs ran)
  // channel pitch of that image: 4 floats past a multiple of 64 floats, so
  // the 16 channels of one epilogue store land on distinct bank groups
  static constexpr int UPP = rup(TPXD, 64) + 4;
  static_assert(!UPS || CIN * UPP * 4 <= XREG, "fused upsample: dX tile does not fit the X region");
  // UPS epilogue items: IKU consecutive source pixels of one source row
  static constexpr int WSU = W / 2, IKU = WSU % 4 == 0 ? 4 : (WSU % 2 == 0 ? 2 : 1), WQU = WSU / IKU;
  static constexpr int NOU = UPS ? CIN * (RT / 2) * WQU : 0, NOI = NOU > 0 ? ceil_div(NOU, 256) : 1;
  // the epilogue's ReLU' mask (flags & 2) is loaded before the next tile's
  // prefetch is issued, so its latency hides behind the tile's MFMAs instead
  // of stalling the epilogue (MW x NTD float4 per lane; UPS: NOI items)
  static constexpr bool AUXP =
      PAIG_BWD_AUXP && (UPS || (VEC4 && MW * NTD <= 8)) && sbwd_auxp(CIN, COUT, H, PM, UPS, PF);
};

template <int CIN, int COUT, int H, int W, int KS, bool UPS, int PM, bool PF>
__global__ void __launch_bounds__(256, (SBwdCfg<CIN, COUT, H, W, KS, UPS, PM, PF>::MINW))
conv_bwd_split_k(FView x, FView dy, FViewW dx, FView aux, const float* __restrict__ w, int flags,
                 float* __restrict__ slab, int F, int ntiles, XMax xm, const s16x8* __restrict__ wp, FView dpool,
                 const unsigned char* __restrict__ pcode, long long pcode_fs) {
  using C = SBwdCfg<CIN, COUT, H, W, KS, UPS, PM, PF>;
  constexpr int KK = C::KK, PADL = C::PADL, RT = C::RT, FPT = C::FPT, ROWS = C::ROWS, TPXV = C::TPXV;
  constexpr int EXT = C::EXT, RTD = C::RTD, ROWSD = C::ROWSD, TPXD = C::TPXD;
  constexpr int CCD = C::CCD, PSD = C::PSD, RPD = C::RPD, KC = C::KC, NS = C::NS, NTD = C::NTD, MW = C::MW;
  constexpr int CQ = C::CQ, NQ = C::NQ, NTX = C::NTX, OFFX = C::OFFX, TWX = C::TWX, XPL = C::XPL;
  constexpr int MT = C::MT, NTF = C::NTF, NTR = C::NTR, KB = C::KB, NCOL = C::NCOL, UPX = C::UPX, W2 = C::W2;
  constexpr int NF1 = NTF > 0 ? NTF : 1, NR1 = NTR > 0 ? NTR : 1;
  constexpr int NID = C::NID, NLD = C::NLD, NIX = C::NIX, NLX = C::NLX;
  constexpr long long HW = (long long)H * W;
  constexpr long long XPLANE = UPS ? (long long)(H / 2) * (W / 2) : HW;
  constexpr int NRB = H / RT;
  extern __shared__ __attribute__((aligned(16))) short lds16[];
  short* Dh = lds16;
  short* Dl = Dh + (C::NIMG == 2 ? C::IMGD : 0);
  short* Wh = lds16 + C::NIMG * C::IMGD;
  short* Wl = Wh + (C::NIMG == 2 ? C::WIMG : 0);
  short* Xh = lds16 + C::NIMG * (C::IMGD + C::WIMG);
  short* Xl = Xh + (C::NIMG == 2 ? C::XIMG : 0);
  float* Sl = reinterpret_cast<float*>(reinterpret_cast<char*>(Xh) + C::XREG);   // UPS window
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, g = lane >> 4;
  __shared__ float smax[4];
#ifdef PAIG_BWD_STAMPS
  unsigned long long st_acc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, st_last = __builtin_amdgcn_s_memtime(), st_n = 0;
#endif

  auto xplane = [](int cq) { return cq * XPL + ((cq & 1) ? 16 : 0) + ((cq & 2) ? 64 : 0); };
  // ---- zero what the staging never writes: the dY image's halo columns,
  // its zero / spare slots, the X image's halo columns
  for (int i = tid; i < FPT * ROWSD * 2 * PADL * CCD; i += 256) {
    const int cc = i % CCD, hc = (i / CCD) % (2 * PADL), r = i / (CCD * 2 * PADL);
    const int xc = hc < PADL ? hc : W + hc;
    const int o = (r * RPD + xc * PSD + cc) * 8;
    *reinterpret_cast<s16x8*>(Dh + o) = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (PM != 2) *reinterpret_cast<s16x8*>(Dl + o) = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  if (tid < 2) {
    *reinterpret_cast<s16x8*>(Dh + (C::ZSLOT + tid) * 8) = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (PM != 2) *reinterpret_cast<s16x8*>(Dl + (C::ZSLOT + tid) * 8) = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  // (UPS: again at every tile's staging -- the epilogue parks the tile's
  // full-resolution dX over the X image, halo columns included)
  auto zero_xhalo = [&]() {
    for (int i = tid; i < FPT * ROWS * 2 * OFFX * CQ; i += 256) {
      const int cq = i % CQ, hc = (i / CQ) % (2 * OFFX), r = i / (CQ * 2 * OFFX);
      const int xc = hc < OFFX ? hc : W + hc;
      *reinterpret_cast<s16x4*>(Xh + xplane(cq) + (r * TWX + xc) * 4) = s16x4{0, 0, 0, 0};
      if (PM != 2) *reinterpret_cast<s16x4*>(Xl + xplane(cq) + (r * TWX + xc) * 4) = s16x4{0, 0, 0, 0};
    }
  };
  zero_xhalo();

  // ---- scales (PM 0): X per launch (ecx), dY per tile (ecd), the
  // data-gradient weights per output channel (ewn)
  int ecx = PAIG_A_EXP, ecd = PM == 0 && PAIG_SCALE_MODE < 2 ? 100 : 0;
  float xsc = 1.f, dsc = __builtin_amdgcn_ldexpf(1.f, ecd);
  float rmax = 0.f;   // range guard (fixed X scale without xmax slots)
  int ewn[NTD];
#pragma unroll
  for (int nt = 0; nt < NTD; ++nt) ewn[nt] = 0;

  // ---- data-gradient weights in fragment order ([s][nt][lane][8]): the
  // layer's transposed + flipped weights (dgrad image of paig_conv_wprep, or
  // staged here from w)
  auto wval = [&](int idx, int j) {
    const int ln = idx & 63, snt = idx >> 6, nt = snt % NTD, s = snt / NTD;
    const int kc = 4 * s + (ln >> 4), ci = nt * 16 + (ln & 15);
    float v = 0.f;
    if (kc < KC && ci < CIN) {
      const int tap = kc / CCD, co = (kc % CCD) * 8 + j;
      if (co < COUT) v = w[(co * CIN + ci) * KK + (KK - 1 - tap)];
    }
    return v;
  };
  __shared__ int sew[PM == 0 ? NTD * 16 : 1];
  if (PM == 0 && wp != nullptr) {
    const int* hdr = reinterpret_cast<const int*>(wp);
    constexpr int HDR = NTD * 16 * 4 / 16;
#pragma unroll
    for (int nt = 0; nt < NTD; ++nt) ewn[nt] = hdr[nt * 16 + (lane & 15)];
    const s16x8* img = wp + HDR;
    constexpr int WLO = NS * NTD * 64;
    for (int idx = tid; idx < NS * NTD * 64; idx += 256) {
      *reinterpret_cast<s16x8*>(Wh + idx * 8) = img[idx];
      *reinterpret_cast<s16x8*>(Wl + idx * 8) = img[WLO + idx];
    }
  } else {
    if constexpr (PM == 0) {
      for (int i = tid; i < NTD * 16; i += 256) sew[i] = 0;
      __syncthreads();
      float pm[NTD];
#pragma unroll
      for (int nt = 0; nt < NTD; ++nt) pm[nt] = 0.f;
      for (int idx = tid; idx < NS * NTD * 64; idx += 256) {
        const int nt = (idx >> 6) % NTD;
#pragma unroll
        for (int j = 0; j < 8; ++j) pm[nt] = fmaxf(pm[nt], fabsf(wval(idx, j)));
      }
#pragma unroll
      for (int nt = 0; nt < NTD; ++nt) atomicMax(&sew[nt * 16 + (tid & 15)], __builtin_bit_cast(int, pm[nt]));
      __syncthreads();
      for (int i = tid; i < NTD * 16; i += 256) sew[i] = f16_scale_exp_v(__builtin_bit_cast(float, sew[i]));
      __syncthreads();
#pragma unroll
      for (int nt = 0; nt < NTD; ++nt) ewn[nt] = sew[nt * 16 + (lane & 15)];
    }
    for (int idx = tid; idx < NS * NTD * 64; idx += 256) {
      const int cl = ((idx >> 6) % NTD) * 16 + (idx & 15);
      const int e = PM == 0 ? sew[cl] : 0;
      s16x8 vh, vl;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        short h, l;
        float rm = 0.f;
        split<PM>(__builtin_amdgcn_ldexpf(wval(idx, j), e), h, l, rm);
        vh[j] = h;
        vl[j] = l;
      }
      *reinterpret_cast<s16x8*>(Wh + idx * 8) = vh;
      if (PM != 2) *reinterpret_cast<s16x8*>(Wl + idx * 8) = vl;
    }
  }

  // ---- data-gradient fragment offsets (slots): pixel base per M-tile,
  // (tap, chunk) per k-step
  int pbase[MW];
#pragma unroll
  for (int mt = 0; mt < MW; ++mt) {
    int pix = (wv * MW + mt) * 16 + (lane & 15);
    if (pix >= TPXD) pix = 0;   // padding rows of the last M-tile: finite data, never stored
    const int fi = pix / (RTD * W), rem = pix % (RTD * W);
    pbase[mt] = (fi * ROWSD + rem / W) * RPD + (rem % W) * PSD;
  }
  int soff[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    int kc = 4 * s + g;
    if (kc >= KC) kc = 0;   // zero weights there
    const int tap = kc / CCD, cc = kc % CCD;
    soff[s] = (tap / KS) * RPD + (tap % KS) * PSD + cc;
  }
  // ---- weight-gradient transposed-read addressing: lane 4q + pl of its
  // 16-lane group supplies row q (pixel 8g + 4h + q of the k-block) of
  // column quad pl
  const int qq = (lane >> 2) & 3, pl = lane & 3;
  auto colt_of = [&](int nt) {
    int cq = nt * 4 + pl;
    if (cq >= NQ) cq = 0;   // padded columns: finite data, never stored
    const int tap = cq / CQ, ciq = cq % CQ;
    return xplane(ciq) + ((tap / KS) * TWX + tap % KS) * 4;
  };
  int colt[NF1], coltr[NR1];
#pragma unroll
  for (int jn = 0; jn < NTF; ++jn) colt[jn] = colt_of(wv + jn * 4);
#pragma unroll
  for (int t = 0; t < NTR; ++t) coltr[t] = colt_of(NTF * 4 + t);
  // dY slot of tile pixel j (its centre position in the halo'd image); the
  // zero slot past the valid pixels
  auto dslot = [&](int j) {
    if (TPXV % 32 != 0 && j >= TPXV) return C::ZSLOT;
    const int fi = j / (RT * W), rem = j % (RT * W);
    return (fi * ROWSD + rem / W + PADL + EXT) * RPD + (rem % W + PADL) * PSD;
  };
  auto xpos = [&](int j) {   // X image position of tile pixel j at tap (0, 0)
    if (TPXV % 32 != 0 && j >= TPXV) j = 0;   // its dY is zero
    const int fi = j / (RT * W), rem = j % (RT * W);
    return ((fi * ROWS + rem / W) * TWX + rem % W + (OFFX - PADL)) * 4;
  };

  f32x4 accw[MT][NF1], accr[MT][NR1];   // whole N-tiles, tail N-tiles (this wave's k-blocks)
#pragma unroll
  for (int m = 0; m < MT; ++m) {
#pragma unroll
    for (int j = 0; j < NF1; ++j) accw[m][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < NR1; ++t) accr[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  float bacc[NLD][8];   // bias partials of this thread's dY units (centre rows), unscaled fp32
#pragma unroll
  for (int l = 0; l < NLD; ++l)
#pragma unroll
    for (int c = 0; c < 8; ++c) bacc[l][c] = 0.f;

  // ---- staging.  dY unit i = (frame fi, image row r, chunk cc, pixel xp),
  // prefetched a tile ahead; X unit i = (fi, r, quad cq, xp)
  float2 pd[NLD][8];
  float2 px[C::XPIPE ? NLX : 1][4];
  // PF: the pooled gradient of each unit's window (8 channels) and the 8
  // window codes (ReLU' bits + argmax, written by the forward's fused pool)
  float dpv[PF ? NLD : 1][8];
  uint2 pcv[PF ? NLD : 1];
  constexpr int HP = H / 2, WP = W / 2;
  using UP = UpStage<UPS ? CIN : 1, H, W, FPT, RT>;
  UP up;
  auto load_d = [&](int t) {
    const int f0 = (t / NRB) * FPT, y0 = (t % NRB) * RT;
    const float* fb = dy.frame(f0 < F ? f0 : 0);
#pragma unroll
    for (int l = 0; l < NLD; ++l) {
      const int i = tid + l * 256;
      const int xp = UPX * (i % W2), r = (i / W2) % ROWSD, cc = (i / (W2 * ROWSD)) % CCD, fi = i / (W2 * ROWSD * CCD);
      const int gy = y0 + r - PADL - EXT;
#ifdef PAIG_BWD_NOLOAD   // diagnostic builds only (wrong results): dY reads from a hot zero buffer
      const bool ok = false;
#else
      const bool ok = i < NID && f0 + fi < F && gy >= 0 && gy < H;
#endif
      const int off = fi * (int)dy.fs + cc * 8 * (int)HW + gy * W + xp;
      static_assert(8 * HW <= 8 * 4096, "paig_zero_planes covers the unit");
      const float* base = ok ? fb + off : paig_zero_planes;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const float* q = COUT % 8 == 0 || cc * 8 + c < COUT ? base + c * (int)HW : paig_zeros;
        pd[l][c] = UPX == 2 ? *reinterpret_cast<const float2*>(q) : make_float2(*q, 0.f);
      }
      if constexpr (PF) {
        const int pw = (gy >> 1) * WP + (xp >> 1);
        const float* pb = ok ? dpool.frame(f0) + fi * (int)dpool.fs + cc * 8 * (HP * WP) + pw : paig_zero_planes;
#pragma unroll
        for (int c = 0; c < 8; ++c) dpv[l][c] = pb[c * (HP * WP)];
        const unsigned char* cb = ok ? pcode + (long long)(f0 + fi) * pcode_fs + ((long long)cc * HP * WP + pw) * 8
                                     : reinterpret_cast<const unsigned char*>(paig_zeros);
        pcv[l] = *reinterpret_cast<const uint2*>(cb);
      }
    }
  };
  // PF: the max pool's backward on the prefetched dY of tile t (before its
  // max and staging): dY = ReLU'(y) * (dY + [pixel is the window's argmax] *
  // d pooled) -- aten max_pool2d backward + the ReLU' of this layer's output,
  // in maxpool_bwd_relu's arithmetic order
  auto fold = [&](int t) {
    const int y0 = (t % NRB) * RT;
#pragma unroll
    for (int l = 0; l < NLD; ++l) {
      const int i = tid + l * 256;
      const int r = (i / W2) % ROWSD;
      const int pr = ((y0 + r - PADL - EXT) & 1) * 2;   // window row of this unit: bits pr, pr + 1
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const unsigned b = ((c < 4 ? pcv[l].x : pcv[l].y) >> (8 * (c & 3))) & 255u;
        const int am = (int)(b >> 4) & 3;
        const float vx = pd[l][c].x + (am == pr ? dpv[l][c] : 0.f);
        const float vy = pd[l][c].y + (am == pr + 1 ? dpv[l][c] : 0.f);
        pd[l][c].x = (b >> pr) & 1u ? vx : 0.f;
        pd[l][c].y = (b >> (pr + 1)) & 1u ? vy : 0.f;
      }
    }
  };
  auto load_x = [&](int t, int i, float2* v) {
    const int f0 = (t / NRB) * FPT, y0 = (t % NRB) * RT;
    const int xp = UPX * (i % W2), r = (i / W2) % ROWS, cq = (i / (W2 * ROWS)) % CQ, fi = i / (W2 * ROWS * CQ);
    const int gy = y0 + r - PADL;
    const bool ok = i < NIX && f0 + fi < F && gy >= 0 && gy < H;
    const float* fb = x.frame(f0 < F ? f0 : 0);
    const int off = fi * (int)x.fs + cq * 4 * (int)XPLANE + gy * W + xp;
    const float* base = ok ? fb + off : paig_zero_planes;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float* q = CIN % 4 == 0 || cq * 4 + c < CIN ? base + c * (int)XPLANE : paig_zeros;
      v[c] = UPX == 2 ? *reinterpret_cast<const float2*>(q) : make_float2(*q, 0.f);
    }
  };
  auto issue = [&](int t) {
    load_d(t);
    if constexpr (UPS) {
      up.issue(x, F, (t / NRB) * FPT, (t % NRB) * RT, tid);
    } else if constexpr (C::XPIPE) {
#pragma unroll
      for (int l = 0; l < NLX; ++l) load_x(t, tid + l * 256, px[l]);
    }
  };
  auto put_d = [&](int i, const float2* v) {
    const int xp = UPX * (i % W2), r = (i / W2) % ROWSD, cc = (i / (W2 * ROWSD)) % CCD, fi = i / (W2 * ROWSD * CCD);
    const int o = ((fi * ROWSD + r) * RPD + (xp + PADL) * PSD + cc) * 8;
    s16x8 h0, l0, h1, l1;
    if constexpr (PM == 0) {
      pf32x2 sv[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) sv[c] = pf32x2{v[c].x, v[c].y} * dsc;
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
      float rm = 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        short h, lo;
        split<PM>(v[c].x, h, lo, rm);
        h0[c] = h;
        l0[c] = lo;
        split<PM>(v[c].y, h, lo, rm);
        h1[c] = h;
        l1[c] = lo;
      }
    }
    *reinterpret_cast<s16x8*>(Dh + o) = h0;
    if (PM != 2) *reinterpret_cast<s16x8*>(Dl + o) = l0;
    if constexpr (UPX == 2) {
      *reinterpret_cast<s16x8*>(Dh + o + PSD * 8) = h1;
      if (PM != 2) *reinterpret_cast<s16x8*>(Dl + o + PSD * 8) = l1;
    }
  };
  auto put_x = [&](int i, const float2* v) {
    const int xp = UPX * (i % W2), r = (i / W2) % ROWS, cq = (i / (W2 * ROWS)) % CQ, fi = i / (W2 * ROWS * CQ);
    const int o = xplane(cq) + ((fi * ROWS + r) * TWX + xp + OFFX) * 4;
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
    if constexpr (UPX == 2) {
      *reinterpret_cast<s16x8*>(Xh + o) = hv;
      if (PM != 2) *reinterpret_cast<s16x8*>(Xl + o) = lv;
    } else {
      *reinterpret_cast<s16x4*>(Xh + o) = s16x4{hv[0], hv[1], hv[2], hv[3]};
      if (PM != 2) *reinterpret_cast<s16x4*>(Xl + o) = s16x4{lv[0], lv[1], lv[2], lv[3]};
    }
  };
  // this wave's max |dY| of the prefetched tile into smax[wv] (before the
  // loop-top barrier; the commit after it reads the block max)
  auto tile_max = [&]() {
    float m = 0.f;
#pragma unroll
    for (int l = 0; l < NLD; ++l)
#pragma unroll
      for (int c = 0; c < 8; ++c) m = amax2(m, pd[l][c].x, pd[l][c].y);
    m = wave_max_u(m);
    if (lane == 0) smax[wv] = m;
  };
  auto commit = [&](int t) {
    if constexpr (PM == 0 && PAIG_SCALE_MODE < 2) {
      // every tile is staged at its own exponent (its max into [2^14, 2^15):
      // the data gradient of a small-gradient tile keeps full precision);
      // the weight-gradient accumulators, held at scale 2^(ecx + ecd), follow
      // exactly (powers of two).  An exponent rise is capped at 2^64 per tile
      // so that rescaled accumulators cannot overflow (tiles 2^64 smaller
      // than the ones before are staged at a lower scale instead)
      const int te = f16_scale_exp(fmaxf(fmaxf(smax[0], smax[1]), fmaxf(smax[2], smax[3])));
      const int td = te < ecd + 64 ? te : ecd + 64;
      if (td != ecd) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
#pragma unroll
            for (int j = 0; j < NF1; ++j) accw[m][j][r] = __builtin_amdgcn_ldexpf(accw[m][j][r], td - ecd);
#pragma unroll
            for (int t = 0; t < NR1; ++t) accr[m][t][r] = __builtin_amdgcn_ldexpf(accr[m][t][r], td - ecd);
          }
        ecd = td;
        dsc = __builtin_amdgcn_ldexpf(1.f, ecd);
      }
    }
    const int f0 = (t / NRB) * FPT;
#pragma unroll
    for (int l = 0; l < NLD; ++l) {
      const int i = tid + l * 256;
      if (NID % 256 != 0 && i >= NID) break;
      put_d(i, pd[l]);
      // bias partials: the tile's own rows (not the halo), frames < F
      const int r = (i / W2) % ROWSD, fi = i / (W2 * ROWSD * CCD);
      if (r >= PADL + EXT && r < PADL + EXT + RT && f0 + fi < F) {
#pragma unroll
        for (int c = 0; c < 8; ++c) bacc[l][c] += pd[l][c].x + pd[l][c].y;
      }
    }
    PAIG_BSTAMP(8);
    if constexpr (UPS) {
      // the half-resolution window (prefetched) -> LDS, then the upsampled
      // rows: units of 4 pixels x 4 channels (one row4 per channel: shared
      // taps and source reads), stored as two 2-pixel staging units
      const int y0 = (t % NRB) * RT;
      up.commit(Sl, tid);
      zero_xhalo();
      PAIG_BSTAMP(9);
      __syncthreads();
      PAIG_BSTAMP(10);
      if constexpr (W % 4 == 0 && ROWS % 2 == 0 && PAIG_BWD_UPS2 && PM == 0 && H != 36) {   // (spills there)
        // items of 4 pixels x 4 channels x a ROW PAIR (image rows 2rp, 2rp+1:
        // output rows y0 - 1 + 2rp (odd) and y0 + 2rp, which interpolate the
        // same two source rows): half the items of the one-row form, each
        // sharing its row reads and horizontal interpolations (c10: 160 items,
        // one pass of the block instead of 320 in one and a quarter passes)
        constexpr int W4 = W / 4, RP2 = ROWS / 2;
#pragma unroll 1
        for (int i = tid; i < CQ * RP2 * W4; i += 256) {
          const int q = i % W4, rp = (i / W4) % RP2, cq = i / (W4 * RP2);
          const int gy = y0 + 2 * rp - PADL;
          const bool ok0 = f0 < F && gy >= 0 && gy < H, ok1 = f0 < F && gy + 1 >= 0 && gy + 1 < H;
          f32x4 o0[4], o1[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            if (cq * 4 + c < CIN) {
              UP::row4x2(Sl, 0, cq * 4 + c, gy, y0, q, ok0, ok1, o0[c], o1[c]);
            } else {
              o0[c] = f32x4{0.f, 0.f, 0.f, 0.f};
              o1[c] = o0[c];
            }
          }
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {
            const int ia = (cq * ROWS + 2 * rp + h2) * W2 + 2 * q;
            const f32x4* o = h2 ? o1 : o0;
            float2 v[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) v[c] = make_float2(o[c][0], o[c][1]);
            put_x(ia, v);
#pragma unroll
            for (int c = 0; c < 4; ++c) v[c] = make_float2(o[c][2], o[c][3]);
            put_x(ia + 1, v);
          }
        }
        PAIG_BSTAMP(11);
      } else if constexpr (W % 4 == 0) {
        constexpr int W4 = W / 4;
#pragma unroll 1
        for (int i = tid; i < NIX / 2; i += 256) {
#ifdef PAIG_BWD_NOUPS   // diagnostic builds only (wrong results): no upsampled X staging
          if (i >= 0) break;
#endif
          const int q = i % W4, r = (i / W4) % ROWS, cq = (i / (W4 * ROWS)) % CQ;
          const int gy = y0 + r - PADL;
          const bool ok = f0 < F && gy >= 0 && gy < H;
          f32x4 o[4];
#pragma unroll
          for (int c = 0; c < 4; ++c)
            o[c] = (ok && cq * 4 + c < CIN) ? UP::row4(Sl, 0, cq * 4 + c, gy, y0, q) : f32x4{0.f, 0.f, 0.f, 0.f};
          const int ia = (cq * ROWS + r) * W2 + 2 * q;
          float2 v[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) v[c] = make_float2(o[c][0], o[c][1]);
          put_x(ia, v);
#pragma unroll
          for (int c = 0; c < 4; ++c) v[c] = make_float2(o[c][2], o[c][3]);
          put_x(ia + 1, v);
        }
        PAIG_BSTAMP(11);
      } else {
        // 3bp's 18-wide c7 (a 9-wide source): one 2-pixel staging unit per item
#pragma unroll 1
        for (int i = tid; i < NIX; i += 256) {
          const int xp = UPX * (i % W2), r = (i / W2) % ROWS, cq = (i / (W2 * ROWS)) % CQ;
          const int gy = y0 + r - PADL;
          const bool ok = f0 < F && gy >= 0 && gy < H;
          float2 v[4];
#pragma unroll
          for (int c = 0; c < 4; ++c)
            v[c] = (ok && cq * 4 + c < CIN)
                       ? make_float2(UP::px1(Sl, 0, cq * 4 + c, gy, y0, xp), UP::px1(Sl, 0, cq * 4 + c, gy, y0, xp + 1))
                       : make_float2(0.f, 0.f);
          put_x(i, v);
        }
      }
    } else if constexpr (C::XPIPE) {
#pragma unroll
      for (int l = 0; l < NLX; ++l) {
        const int i = tid + l * 256;
        if (NIX % 256 != 0 && i >= NIX) break;
        put_x(i, px[l]);
      }
    } else {
#pragma unroll 1
      for (int i = tid; i < NIX; i += 256) {
        float2 v[4];
        load_x(t, i, v);
        put_x(i, v);
      }
    }
  };

  int lt = blockIdx.x;
  auto tile_of = [&](int l) { return l < ntiles ? xcd_tile(l, ntiles) : ntiles; };
  issue(tile_of(lt));
  if (PM == 0 && xm.p) {
    // the launch's X exponent: max over the forward's per-block slots
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
    __syncthreads();
  }
  if constexpr (PM == 0) xsc = __builtin_amdgcn_ldexpf(1.f, ecx);
  else ecx = 0;

  PAIG_BSTAMP(0);
  for (; lt < ntiles; lt += gridDim.x) {
    const int tile = xcd_tile(lt, ntiles);
    const int f0 = (tile / NRB) * FPT, y0 = (tile % NRB) * RT;
    if constexpr (PF) fold(tile);
    if constexpr (PM == 0 && PAIG_SCALE_MODE < 2) tile_max();
    __syncthreads();   // the previous tile's fragment reads are done
    PAIG_BSTAMP(1);
    commit(tile);
    __syncthreads();
    PAIG_BSTAMP(2);
    // this tile's ReLU' mask for the epilogue (AUXP), issued before the next
    // tile's prefetch: the epilogue then waits for it alone
    typedef float fIKU __attribute__((ext_vector_type(C::IKU)));
    f32x4 auxv[C::AUXP && !UPS ? MW : 1][C::AUXP && !UPS ? NTD : 1];
    fIKU auxu[C::AUXP && UPS ? C::NOI : 1];
    if constexpr (C::AUXP) {
      if (flags & 2) {
        if constexpr (UPS) {
#pragma unroll
          for (int k = 0; k < C::NOI; ++k) {
            const int o = tid + 256 * k;
            const int q = o % C::WQU, sr = (o / C::WQU) % (RT / 2), ci = o / (C::WQU * (RT / 2));
            const bool ok = o < C::NOU && f0 < F;
            const float* ap = ok ? aux.frame(f0) + ((long long)ci * (H / 2) + y0 / 2 + sr) * C::WSU + C::IKU * q
                                 : paig_zero_planes;
            auxu[k] = *reinterpret_cast<const fIKU*>(ap);
          }
        } else {
#pragma unroll
          for (int nt = 0; nt < NTD; ++nt) {
            const int ci = nt * 16 + (lane & 15);
#pragma unroll
            for (int mt = 0; mt < MW; ++mt) {
              const int pix = (wv * MW + mt) * 16 + (lane >> 4) * 4;
              const int fi = pix / (RT * W), rem = pix % (RT * W);
              const int f = f0 + fi;
              const bool ok = ci < CIN && pix < TPXV && f < F;
              const float* ap = ok ? aux.frame(f) + ci * HW + (long long)(y0 + rem / W) * W + rem % W
                                   : paig_zero_planes;
              auxv[mt][nt] = *reinterpret_cast<const f32x4*>(ap);
            }
          }
        }
      }
    }
    issue(tile_of(lt + gridDim.x));
    PAIG_BSTAMP(3);

    // ---- weight gradient: all 4 waves over all k-blocks, each its whole
    // N-tiles; the tail N-tiles over every 4th k-block
#pragma unroll 2
    for (int kb = 0; kb < KB; ++kb) {
      const int p0 = kb * 32;
      s16x8 ah[MT], al[MT];
      const int d0 = dslot(p0 + 8 * g + qq), d1 = dslot(p0 + 8 * g + 4 + qq);
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        // channels 16m + 4pl .. +3: chunk 2m + pl/2, half pl%2 (rows co >=
        // COUT read finite neighbouring data and are discarded)
        const int co = 2 * m + (pl >> 1), hoff = (pl & 1) * 4;
        const int a0 = (d0 + co) * 8 + hoff, a1 = (d1 + co) * 8 + hoff;
        ah[m] = __builtin_shufflevector(tr_read(Dh + a0), tr_read(Dh + a1), 0, 1, 2, 3, 4, 5, 6, 7);
        al[m] = PM != 2 ? __builtin_shufflevector(tr_read(Dl + a0), tr_read(Dl + a1), 0, 1, 2, 3, 4, 5, 6, 7) : ah[m];
      }
      const int r0 = xpos(p0 + 8 * g + qq), r1 = xpos(p0 + 8 * g + 4 + qq);
      auto ntile = [&](int ct, f32x4* acc) __attribute__((always_inline)) {
        const s16x8 bh = __builtin_shufflevector(tr_read(Xh + r0 + ct), tr_read(Xh + r1 + ct), 0, 1, 2, 3, 4, 5, 6, 7);
        const s16x8 bl =
            PM != 2 ? __builtin_shufflevector(tr_read(Xl + r0 + ct), tr_read(Xl + r1 + ct), 0, 1, 2, 3, 4, 5, 6, 7) : bh;
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m] = mma3<PM>(ah[m], al[m], bh, bl, acc[m]);
      };
#pragma unroll
      for (int jn = 0; jn < NTF; ++jn) {
        if (!C::BAL && wv + jn * 4 >= NTX) continue;   // wave-uniform
        f32x4 a[MT];
#pragma unroll
        for (int m = 0; m < MT; ++m) a[m] = accw[m][jn];
        ntile(colt[jn], a);
#pragma unroll
        for (int m = 0; m < MT; ++m) accw[m][jn] = a[m];
      }
      if (NTR > 0 && (kb & 3) == wv) {   // wave-uniform: EXEC stays full for the transposed reads
#pragma unroll
        for (int t = 0; t < NTR; ++t) {
          f32x4 a[MT];
#pragma unroll
          for (int m = 0; m < MT; ++m) a[m] = accr[m][t];
          ntile(coltr[t], a);
#pragma unroll
          for (int m = 0; m < MT; ++m) accr[m][t] = a[m];
        }
      }
    }

    PAIG_BSTAMP(4);
    // ---- data gradient of the tile's pixels
    f32x4 accd[MW][NTD];
#pragma unroll
    for (int mt = 0; mt < MW; ++mt)
#pragma unroll
      for (int nt = 0; nt < NTD; ++nt) accd[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      s16x8 bh[NTD], bl[NTD];
#pragma unroll
      for (int nt = 0; nt < NTD; ++nt) {
        const int o = ((s * NTD + nt) * 64 + lane) * 8;
        bh[nt] = *reinterpret_cast<const s16x8*>(Wh + o);
        bl[nt] = PM != 2 ? *reinterpret_cast<const s16x8*>(Wl + o) : bh[nt];
      }
#pragma unroll
      for (int mt = 0; mt < MW; ++mt) {
        const int o = (pbase[mt] + soff[s]) * 8;
        const s16x8 ah = *reinterpret_cast<const s16x8*>(Dh + o);
        const s16x8 al = PM != 2 ? *reinterpret_cast<const s16x8*>(Dl + o) : ah;
#pragma unroll
        for (int nt = 0; nt < NTD; ++nt) accd[mt][nt] = mma3<PM>(ah, al, bh[nt], bl[nt], accd[mt][nt]);
      }
    }
    PAIG_BSTAMP(5);
    if constexpr (UPS) {
      // full-resolution dX rows y0-1 .. y0+RT of the tile -> LDS [ci][RTD][W]
      // (the X image is free once every wave's weight-gradient reads are done)
      float* U = reinterpret_cast<float*>(Xh);
      __syncthreads();
#pragma unroll
      for (int nt = 0; nt < NTD; ++nt) {
        const int ci = nt * 16 + (lane & 15);
        if (ci >= CIN) continue;
        const float tinv = PM == 0 ? __builtin_amdgcn_ldexpf(1.f, -(ecd + ewn[nt])) : 1.f;
#pragma unroll
        for (int mt = 0; mt < MW; ++mt) {
          const int pix = (wv * MW + mt) * 16 + (lane >> 4) * 4;
          if (pix < TPXD) *reinterpret_cast<f32x4*>(U + ci * C::UPP + pix) = accd[mt][nt] * tinv;
        }
      }
      __syncthreads();
      // the 2x bilinear upsample's transpose (aten upsample_bilinear2d
      // backward, align_corners=False: source s gets outputs 2s-1 .. 2s+2
      // with weights 1/4, 3/4, 3/4, 1/4; 1 at the clamped edges), in
      // upsample_bwd_k's per-pixel order; then ReLU' of the source and the
      // store.  Item = IK (4; 2 or 1 where the source width is not a multiple
      // of 4: 3bp's 18 / 9) consecutive source pixels of one row: full-resolution
      // columns 2 IK q - 1 .. 2 IK q + 2 IK of 4 rows
      constexpr int HS = H / 2, WS = W / 2, IK = C::IKU, WQ = C::WQU;
      constexpr int NO = C::NOU;
      static_assert(WS % IK == 0, "IK-pixel source items");
      typedef fIKU fIK;
      // item o; mp: its prefetched ReLU' mask (AUXP)
      auto item = [&](int o, const fIK& mp) __attribute__((always_inline)) {
        const int q = o % WQ, sr = (o / WQ) % (RT / 2), ci = o / (WQ * (RT / 2));
        const int sy = y0 / 2 + sr;
        float wy[4];
        wy[0] = sy >= 1 ? 0.25f : 0.f;
        wy[1] = sy == 0 ? 1.f : 0.75f;
        wy[2] = sy == HS - 1 ? 1.f : 0.75f;
        wy[3] = sy <= HS - 2 ? 0.25f : 0.f;
        fIK acc;
#pragma unroll
        for (int k = 0; k < IK; ++k) acc[k] = 0.f;
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          // full row 2sy - 1 + a = tile dX row 2sr + a (row 0 = y0 - 1)
          if (wy[a] == 0.f) continue;
          const float* rp = U + ci * C::UPP + (2 * sr + a) * W + 2 * IK * q;
          float c[2 * IK + 2];
          c[0] = q > 0 ? rp[-1] : 0.f;
          c[2 * IK + 1] = q < WQ - 1 ? rp[2 * IK] : 0.f;
          if constexpr (IK == 1) {
            c[1] = rp[0];
            c[2] = rp[1];
          } else {
#pragma unroll
            for (int h = 0; h < IK / 2; ++h) {
              const f32x4 m = *reinterpret_cast<const f32x4*>(rp + 4 * h);
#pragma unroll
              for (int e = 0; e < 4; ++e) c[1 + 4 * h + e] = m[e];
            }
          }
          // source pixels IK q + k read columns 2 IK q + 2k - 1 .. 2 IK q + 2k + 2
          fIK row;
#pragma unroll
          for (int k = 0; k < IK; ++k) {
            const int sx = IK * q + k;
            float wx[4];
            wx[0] = sx >= 1 ? 0.25f : 0.f;
            wx[1] = sx == 0 ? 1.f : 0.75f;
            wx[2] = sx == WS - 1 ? 1.f : 0.75f;
            wx[3] = sx <= WS - 2 ? 0.25f : 0.f;
            float v = 0.f;
#pragma unroll
            for (int b = 0; b < 4; ++b)
              if (wx[b] != 0.f) v = fmaf(wx[b], c[2 * k + b], v);
            row[k] = v;
          }
#pragma unroll
          for (int k = 0; k < IK; ++k) acc[k] = fmaf(wy[a], row[k], acc[k]);
        }
        if (f0 < F) {
          const long long off = ((long long)ci * HS + sy) * WS + IK * q;
          float* op = dx.frame(f0) + off;
          if (flags & 4) acc += *reinterpret_cast<const fIK*>(op);
          if (flags & 2) {
            fIK m;
            if constexpr (C::AUXP) m = mp;
            else m = *reinterpret_cast<const fIK*>(aux.frame(f0) + off);
#pragma unroll
            for (int k = 0; k < IK; ++k) acc[k] = m[k] > 0.f ? acc[k] : 0.f;
          }
          *reinterpret_cast<fIK*>(op) = acc;
        }
      };
      if constexpr (C::AUXP) {
#pragma unroll
        for (int it = 0; it < C::NOI; ++it) {
          const int o = tid + 256 * it;
          if (NO % 256 != 0 && o >= NO) break;
          item(o, auxu[it]);
        }
      } else {
        for (int o = tid; o < NO; o += 256) item(o, auxu[0]);
      }
    } else {
    // epilogue: lane holds pixels (lane>>4)*4 + r of each M-tile for input
    // channel ci = nt*16 + (lane&15); flags 2: * (aux > 0), 4: accumulate
#pragma unroll
    for (int nt = 0; nt < NTD; ++nt) {
      const int ci = nt * 16 + (lane & 15);
      if (ci >= CIN) continue;
      const float tinv = PM == 0 ? __builtin_amdgcn_ldexpf(1.f, -(ecd + ewn[nt])) : 1.f;
#pragma unroll
      for (int mt = 0; mt < MW; ++mt) {
        const int pix = (wv * MW + mt) * 16 + (lane >> 4) * 4;
        if constexpr (C::VEC4) {
          if (pix >= TPXV) continue;
          const int fi = pix / (RT * W), rem = pix % (RT * W);
          const int y = y0 + rem / W, xx = rem % W, f = f0 + fi;
          if (f >= F) continue;
          float* op = dx.frame(f) + ci * HW + (long long)y * W + xx;
          f32x4 v = accd[mt][nt] * tinv;
          if (flags & 4) v += *reinterpret_cast<const f32x4*>(op);
          if (flags & 2) {
            f32x4 a;
            if constexpr (C::AUXP) a = auxv[mt][nt];
            else a = *reinterpret_cast<const f32x4*>(aux.frame(f) + ci * HW + (long long)y * W + xx);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = a[r] > 0.f ? v[r] : 0.f;
          }
          *reinterpret_cast<f32x4*>(op) = v;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int pr = pix + r;
            if (pr >= TPXV) break;
            const int fi = pr / (RT * W), rem = pr % (RT * W);
            const int y = y0 + rem / W, xx = rem % W, f = f0 + fi;
            if (f >= F) continue;
            float* op = dx.frame(f) + ci * HW + (long long)y * W + xx;
            float v = accd[mt][nt][r] * tinv;
            if (flags & 4) v += *op;
            if (flags & 2) v = aux.frame(f)[ci * HW + (long long)y * W + xx] > 0.f ? v : 0.f;
            *op = v;
          }
        }
      }
    }
    }   // !UPS
    PAIG_BSTAMP(6);
#ifdef PAIG_BWD_STAMPS
    ++st_n;
#endif
  }

  // ---- this block's slab row: weight gradients (each wave its N-tiles,
  // scaled back exactly), then the bias
  float* s = slab + (long long)blockIdx.x * C::SLAB;
  auto put_w = [&](int m, int nt, const f32x4& acc) __attribute__((always_inline)) {
    const int col = nt * 16 + (lane & 15), cq = col >> 2;
    const int tap = cq / CQ, ci = (cq % CQ) * 4 + (col & 3);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = m * 16 + (lane >> 4) * 4 + r;
      float v = acc[r];
      if constexpr (PM == 0) v = __builtin_amdgcn_ldexpf(v, -(ecx + ecd));
      if (co < COUT && cq < NQ && ci < CIN) s[co * NCOL + ci * KK + tap] = v;
    }
  };
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j = 0; j < NTF; ++j)
      if (wv + j * 4 < NTX) put_w(m, wv + j * 4, accw[m][j]);
  if constexpr (NTR > 0) {
    // tail N-tiles: the 4 waves' k-block partials, summed in wave order
    f32x4* Rt = reinterpret_cast<f32x4*>(lds16);   // [4][MT][NTR][64]
    __syncthreads();   // the last tile's LDS reads are done
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int t = 0; t < NTR; ++t) Rt[((wv * MT + m) * NTR + t) * 64 + lane] = accr[m][t];
    __syncthreads();
    for (int u = wv; u < MT * NTR; u += 4) {
      f32x4 v = Rt[u * 64 + lane];
#pragma unroll
      for (int w = 1; w < 4; ++w) v += Rt[(w * MT * NTR + u) * 64 + lane];
      put_w(u / NTR, NTF * 4 + u % NTR, v);
    }
  }
  // bias: unit i of thread i % 256 (slot i / 256) kept the partials of its 8
  // channels.  Two fixed-order stages: thread (channel co, part q) sums the
  // units q, q + NP, ... of co's chunk; thread co then sums its NP parts
  __syncthreads();
  float* Rb = reinterpret_cast<float*>(lds16);   // [NLD][256][8], then [COUT][NP]
  constexpr int NP = 256 / COUT, NU = FPT * ROWSD * W2;   // parts per channel, units per chunk
  float* Rp = Rb + NLD * 256 * 8;
#pragma unroll
  for (int l = 0; l < NLD; ++l)
#pragma unroll
    for (int c = 0; c < 8; ++c) Rb[(l * 256 + tid) * 8 + c] = bacc[l][c];
  __syncthreads();
  if (tid < NP * COUT) {
    const int co = tid % COUT, q = tid / COUT, cc = co / 8, c = co % 8;
    float v = 0.f;
    for (int j = q; j < NU; j += NP) {
      const int xpi = j % W2, r = (j / W2) % ROWSD, fi = j / (W2 * ROWSD);
      v += Rb[((((fi * CCD + cc) * ROWSD) + r) * W2 + xpi) * 8 + c];
    }
    Rp[co * NP + q] = v;
  }
  __syncthreads();
  if (tid < COUT) {
    float v = 0.f;
    for (int q = 0; q < NP; ++q) v += Rp[tid * NP + q];
    s[COUT * NCOL + tid] = v;
  }
  if constexpr (PM == 0) f16_range_note(rmax);
#ifdef PAIG_BWD_STAMPS
  PAIG_BSTAMP(7);
  if (lane == 0 && blockIdx.x < 4096) {
#pragma unroll
    for (int k = 0; k < 12; ++k) paig_bwd_stamps[blockIdx.x][wv][k] = st_acc[k];
    paig_bwd_stamps[blockIdx.x][wv][12] = st_n;
  }
#endif
}

template <int CIN, int COUT, int H, int W, int KS, bool UPS, int PM, bool PF = false>
static int sbwd_launch(FView x, FView dy, FViewW dx, FView aux, const float* w, int flags, float* slab, int nblk_max,
                       int* nblk_out, int F, hipStream_t st, XMax xm, const void* wp,
                       FView dpool = FView{nullptr, 0, 0, 0}, const unsigned char* pcode = nullptr,
                       long long pcode_fs = 0) {
  using C = SBwdCfg<CIN, COUT, H, W, KS, UPS, PM, PF>;
  constexpr int RED = (C::NLD * 256 * 8 + 256) * 4;   // the bias reduction's LDS
  constexpr int LDS0 = C::LDS > RED ? C::LDS : RED;
  static_assert(LDS0 <= LDS_MAX, "fused backward: staging exceeds the LDS");
  // A/B: PAIG_BWD_LDS_PAD = extra bytes of (unused) LDS per block, the
  // occupancy cost an LDS landing zone for the next tile would have
  static const int lds_pad = [] {
    const char* e = getenv("PAIG_BWD_LDS_PAD");
    return e ? atoi(e) : 0;
  }();
  const int LDS = LDS0 + lds_pad <= LDS_MAX ? LDS0 + lds_pad : LDS0;
  const int ntiles = cdiv(F, C::FPT) * (H / C::RT);
  auto k = conv_bwd_split_k<CIN, COUT, H, W, KS, UPS, PM, PF>;
  static int resident = 0;
  if (!resident) {
    if (LDS > 64 * 1024) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    resident = persistent_grid((const void*)k, LDS);
  }
  int nb = ntiles < nblk_max ? ntiles : nblk_max;
  if (nb > resident) nb = resident;
  {
    // A/B: PAIG_BWD_MIN_TPB = minimum tiles per block (fewer slab rows on
    // the layers with few tiles)
    static int mt = -1;
    if (mt < 0) {
      const char* e = getenv("PAIG_BWD_MIN_TPB");
      mt = e ? atoi(e) : 0;
    }
    if (mt > 1 && nb > cdiv(ntiles, mt)) nb = cdiv(ntiles, mt);
  }
  if (nb < 1) nb = 1;
  *nblk_out = nb;
  PAIG_REQUIRE(!xm.p || (xm.n % 4 == 0 && (reinterpret_cast<uintptr_t>(xm.p) & 15) == 0),
               "conv split bwd: xmax needs 16-byte alignment and a multiple of 4 slots (%d)", xm.n);
  PAIG_REQUIRE(!(flags & 2) || aux.p, "conv split bwd: ReLU' mask (flags & 2) without aux");
  PAIG_REQUIRE(!PF || (dpool.p && pcode && (reinterpret_cast<uintptr_t>(pcode) & 7) == 0 && pcode_fs % 8 == 0),
               "conv split bwd: pool fold needs the pooled gradient and 8-byte aligned window codes");
  hipLaunchKernelGGL(k, dim3(nb), dim3(256), LDS, st, x, dy, dx, aux, w, flags, slab, F, ntiles, xm,
                     PM == 0 ? static_cast<const s16x8*>(wp) : nullptr, dpool, pcode, pcode_fs);
  PAIG_CHECK_LAUNCH();
  return 0;
}

// (CIN, COUT, H) of the fused layers: the 3x3 convs with a data gradient
// (every layer but the first) of the ShallowUNet at 32 x 32 (spring,
// bouncing) and 36 x 36 (3bp; its 9 x 9 level keeps the separate kernels:
// odd rows and 32-channel tiles spill registers in the fused form)
// the fused-upsample layers (input = the 2x bilinear upsample of a half-
// resolution source; the upsample's transpose folded into the data gradient)
#define PAIG_BWD_UP_SHAPES(X) X(32, 16, 16) X(16, 16, 32) X(16, 16, 36) X(32, 16, 18)
// the layers whose output feeds a 2x2 max pool fused into their forward
// (c2, c4 of the ShallowUNet): the pool's backward folded into the dY
// staging (flags & 64).  The UNet (mnist) keeps its standalone pools (its
// forward convs have no fused pool at 64 / 32 wide), and of its layers only
// those that measured faster fused are listed (c2, c17: 16 -> 16 at 64 x 64;
// c3: 16 -> 32 at 32 x 32); its wider or 1-block-per-CU shapes (c4 / c14,
// c15's upsample, c16) measured 14-40% slower than the separate kernels
#define PAIG_BWD_POOL_SHAPES(X) X(8, 8, 32) X(16, 16, 16) X(16, 16, 64) X(8, 8, 36) X(16, 16, 18)
#define PAIG_BWD_SHAPES(X)                                                                  \
  X(8, 8, 32) X(8, 16, 16) X(16, 16, 16) X(16, 32, 8) X(32, 32, 8) X(32, 16, 16) X(24, 8, 32) \
  X(8, 8, 36) X(8, 16, 18) X(16, 16, 18) X(32, 16, 18) X(24, 8, 36)                            \
  X(16, 16, 64) X(16, 32, 32)

}  // namespace

extern "C" {

int paig_conv2d_bwd_supported(int Cin, int Cout, int H, int W, int ks, int flags) {
  if (H != W || ks != 3 || !(flags & (128 | 256))) return 0;
#define PAIG_CASE(CI, CO, HH) \
  if (Cin == CI && Cout == CO && H == HH) return 1;
  if (flags & 64) {
    if (flags & 32) return 0;
    PAIG_BWD_POOL_SHAPES(PAIG_CASE)
    return 0;
  }
  if (flags & 32) {
    PAIG_BWD_UP_SHAPES(PAIG_CASE)
    return 0;
  }
  PAIG_BWD_SHAPES(PAIG_CASE)
#undef PAIG_CASE
  return 0;
}

int paig_conv2d_bwd(const float* x, long long x_fs, int x_grp, long long x_gs, const float* dy, long long dy_fs,
                    float* dx, long long dx_fs, const float* aux, long long aux_fs, const float* w, float* slab,
                    int nblk_max, int* nblk_out, int F, int Cin, int Cout, int H, int W, int ks, int flags,
                    const float* xmax, int xmax_n, const float* dpool, long long dpool_fs,
                    const unsigned char* pcode, long long pcode_fs, const void* wprep, void* stream) {
  *nblk_out = 0;
  if (F <= 0) return 0;
  PAIG_REQUIRE(paig_conv2d_bwd_supported(Cin, Cout, H, W, ks, flags),
               "paig_conv2d_bwd: no fused kernel for Cin=%d Cout=%d H=%d W=%d ks=%d flags=%d", Cin, Cout, H, W, ks,
               flags);
  PAIG_REQUIRE(x_grp == 0 || H * W >= 256, "paig_conv2d_bwd: multi-frame tiles need a plain frame stride");
  PAIG_REQUIRE(nblk_max > 0 && slab && dx && dy && x && w, "paig_conv2d_bwd: null operand or no slab rows");
  hipStream_t st = (hipStream_t)stream;
  FView vx{x, x_fs, x_gs, x_grp}, vd{dy, dy_fs, 0, 0}, va{aux, aux_fs, 0, 0};
  FViewW vdx{dx, dx_fs};
  XMax xm{const_cast<float*>(xmax), xmax_n};
  const bool b16 = (flags & 256) != 0;
  const int fl = flags & 6;
  if (flags & 64) {
    const FView vp{dpool, dpool_fs, 0, 0};
#define PAIG_CASE(CI, CO, HH)                                                                                     \
  if (Cin == CI && Cout == CO && H == HH)                                                                         \
    return b16 ? sbwd_launch<CI, CO, HH, HH, 3, false, 2, true>(vx, vd, vdx, va, w, fl, slab, nblk_max, nblk_out,  \
                                                                 F, st, xm, wprep, vp, pcode, pcode_fs)            \
               : sbwd_launch<CI, CO, HH, HH, 3, false, 0, true>(vx, vd, vdx, va, w, fl, slab, nblk_max, nblk_out,  \
                                                                 F, st, xm, wprep, vp, pcode, pcode_fs);
    PAIG_BWD_POOL_SHAPES(PAIG_CASE)
#undef PAIG_CASE
    return PAIG_E_UNSUPPORTED;
  }
  if (flags & 32) {
#define PAIG_CASE(CI, CO, HH)                                                                                     \
  if (Cin == CI && Cout == CO && H == HH)                                                                         \
    return b16 ? sbwd_launch<CI, CO, HH, HH, 3, true, 2>(vx, vd, vdx, va, w, fl, slab, nblk_max, nblk_out, F, st, \
                                                           xm, wprep)                                             \
               : sbwd_launch<CI, CO, HH, HH, 3, true, 0>(vx, vd, vdx, va, w, fl, slab, nblk_max, nblk_out, F, st, \
                                                           xm, wprep);
    PAIG_BWD_UP_SHAPES(PAIG_CASE)
#undef PAIG_CASE
    return PAIG_E_UNSUPPORTED;
  }
#define PAIG_CASE(CI, CO, HH)                                                                                      \
  if (Cin == CI && Cout == CO && H == HH)                                                                          \
    return b16 ? sbwd_launch<CI, CO, HH, HH, 3, false, 2>(vx, vd, vdx, va, w, fl, slab, nblk_max, nblk_out, F, st, \
                                                            xm, wprep)                                             \
               : sbwd_launch<CI, CO, HH, HH, 3, false, 0>(vx, vd, vdx, va, w, fl, slab, nblk_max, nblk_out, F, st, \
                                                            xm, wprep);
  PAIG_BWD_SHAPES(PAIG_CASE)
#undef PAIG_CASE
  return PAIG_E_UNSUPPORTED;
}

#ifdef PAIG_BWD_STAMPS
int paig_bwd_stamps_read(void* host, size_t bytes) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(paig_bwd_stamps), bytes);
}
#endif

}  // extern "C"

PAIG_F16_RANGE_ACCESSOR(paig_f16_range_bwd)
