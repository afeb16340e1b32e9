// fp32 GEMM on CDNA4 matrix cores (v_mfma_f32_16x16x4_f32: exact f32 FMA
// chain, same rate as the f32 VALU but one instruction per 16 FMAs/lane).
//
// Used for every dense layer of the path: the encoder's projection to latent
// coordinates (nn/network/blocks.py:71-75,98-100; K = 3072 -> 200, the one
// MFMA-shaped op the north star names), its MLP tail and the velocity MLP
// (blocks.py:23-29), forward and backward (dX = dY W, dW = dY^T X, and the
// bias gradient db = colsum(dY) fused into the dW GEMM as row sums of op(A)).
//
//   C[M,N] = alpha * op(A)[M,K] op(B)[K,N]  (+ beta*C) (+ bias[n]) -> act -> *aux'
//   op(A)[m][k] = TA ? A[k*lda+m] : A[m*lda+k]
//   op(B)[k][n] = TB ? B[n*ldb+k] : B[k*ldb+n]
//   rowsum[m] = sum_k op(A)[m][k]            (optional)
//
// Tile 64x64x32, 256 threads = 4 waves in 2x2, each wave 32x32 = 2x2 MFMA
// tiles.  Global loads are float4 along each operand's contiguous dimension;
// the LDS image keeps that orientation ([row][k] with pitch 34 = 2 mod 32, or
// [k][row] with pitch 80 = 16 mod 32) so the 16B loads land with wide LDS
// writes AND every MFMA fragment read is bank-conflict free.  The next K
// tile is prefetched into registers while the current one is multiplied.
// Split-K writes fp32 partial slabs reduced by gemm_splitk_epilogue_k
// (deterministic).
#include "common.h"

#include <algorithm>
#include <cstdlib>

namespace {

constexpr int BM = 64, BN = 64, BK = 32;
constexpr int LDRK = BK + 2;    // [row][k] image pitch
constexpr int LDKR = 64 + 16;   // [k][row] image pitch
constexpr int IMG = (BK * LDKR > 64 * LDRK ? BK * LDKR : 64 * LDRK);

typedef float f32x4 __attribute__((ext_vector_type(4)));

// the source of out-of-range operand elements (Tile::load_bf)
__device__ __attribute__((aligned(16))) float zero16[4];   // zero-initialised, never written

// One operand tile (64 rows x BK k) as 2 float4 per thread.
//  KCONTIG: element (r, k) at p[(r0 + r) * ld + k0 + k]   -> image [r][k]
// !KCONTIG: element (r, k) at p[(k0 + k) * ld + r0 + r]   -> image [k][r]
template <bool KCONTIG>
struct Tile {
  f32x4 v[2];
  __device__ __forceinline__ void load(const float* __restrict__ p, long long ld, int r0, int k0, int R, int K,
                                       bool vec, int tid) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      int r, k;
      if (KCONTIG) { r = (tid >> 3) + 32 * e; k = (tid & 7) * 4; }
      else { k = (tid >> 4) + 16 * e; r = (tid & 15) * 4; }
      const int gr = r0 + r, gk = k0 + k;
      f32x4 x = f32x4{0.f, 0.f, 0.f, 0.f};
      if (KCONTIG) {
        if (gr < R) {
          const float* q = p + (long long)gr * ld + gk;
          if (vec && gk + 3 < K) x = *reinterpret_cast<const f32x4*>(q);
          else
#pragma unroll
            for (int i = 0; i < 4; ++i) x[i] = (gk + i < K) ? q[i] : 0.f;
        }
      } else {
        if (gk < K) {
          const float* q = p + (long long)gk * ld + gr;
          if (vec && gr + 3 < R) x = *reinterpret_cast<const f32x4*>(q);
          else
#pragma unroll
            for (int i = 0; i < 4; ++i) x[i] = (gr + i < R) ? q[i] : 0.f;
        }
      }
      v[e] = x;
    }
  }
  // Branch-free form (split kernels): every lane issues its loads, and an
  // out-of-range element reads a zero from zero16 instead (the address is
  // selected, not the data, so nothing waits on the load before its use):
  // the compiler counts the loads in flight and the register ring really
  // overlaps them (branchy or data-selected loads made it wait for all).
  // VEC: float4 along the contiguous dimension, which must then be a multiple
  // of 4 with 16-byte aligned rows.
  template <bool VEC>
  __device__ __forceinline__ void load_bf(const float* __restrict__ p, long long ld, int r0, int k0, int R, int K,
                                          int tid) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      int r, k;
      if (KCONTIG) { r = (tid >> 3) + 32 * e; k = (tid & 7) * 4; }
      else { k = (tid >> 4) + 16 * e; r = (tid & 15) * 4; }
      const int gr = r0 + r, gk = k0 + k;
      if constexpr (VEC) {
        const bool ok = gr < R && gk < K;
        const float* q = ok ? p + (KCONTIG ? (long long)gr * ld + gk : (long long)gk * ld + gr) : zero16;
        v[e] = *reinterpret_cast<const f32x4*>(q);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rr = KCONTIG ? gr : gr + i, kk = KCONTIG ? gk + i : gk;
          const bool ok = rr < R && kk < K;
          v[e][i] = *(ok ? p + (KCONTIG ? (long long)rr * ld + kk : (long long)kk * ld + rr) : zero16);
        }
      }
    }
  }
  __device__ __forceinline__ void store(float* img, int tid) const {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      if (KCONTIG) {
        const int r = (tid >> 3) + 32 * e, k = (tid & 7) * 4;
        float* q = img + r * LDRK + k;
        *reinterpret_cast<float2*>(q) = make_float2(v[e][0], v[e][1]);
        *reinterpret_cast<float2*>(q + 2) = make_float2(v[e][2], v[e][3]);
      } else {
        const int k = (tid >> 4) + 16 * e, r = (tid & 15) * 4;
        *reinterpret_cast<f32x4*>(img + k * LDKR + r) = v[e];
      }
    }
  }
  // fragment element (row, k) of the image
  static __device__ __forceinline__ float at(const float* img, int r, int k) {
    return KCONTIG ? img[r * LDRK + k] : img[k * LDKR + r];
  }
};

// XCD-aware tile order.  Workgroups are dispatched round-robin over the 8
// XCDs (linear id mod 8), each with its own L2.  Logical tiles are renumbered
// so each XCD gets a contiguous run, ordered along the smaller grid dimension
// first: the blocks that re-read one operand tile (the N-tiles of an M-row
// block, or the M-tiles of an N-column block) then share that XCD's L2
// instead of fetching the operand once per XCD.
// A split-K epilogue deferred into the next GEMM launch (paig_gemm_defer_epilogue):
// that launch's grid has one more z-plane whose blocks run it (S = 0: none)
struct PendEpi {
  int M, N, S;
  const float* part;
  float* C;
  long long ldc;
  float beta;
  const float* bias;
  int act, auxm;
  const float* aux;
  long long ldaux;
  const float* rowpart;
  float* rowsum;
  int v4;
};
__device__ void splitk_epi_run(const PendEpi& pe, int bid, int nb);
// (a GEMM kernel's first statement: the deferred epilogue's blocks leave)
#define PAIG_PENDING_EPI(pe)                                                      \
  if ((pe).S && (int)blockIdx.z == (int)gridDim.z - 1) {                          \
    splitk_epi_run((pe), blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y); \
    return;                                                                      \
  }

struct TileId {
  int x, y, z;
};
// gz: the GEMM's own z-planes (a deferred epilogue's plane excluded)
__device__ __forceinline__ TileId xcd_tile(int gz) {
  const int nx = gridDim.x, ny = gridDim.y, total = nx * ny * gz;
  int lin = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z);
  if (total % 8 == 0) lin = (lin % 8) * (total / 8) + lin / 8;
  TileId t;
  if (nx <= ny) {
    t.x = lin % nx;
    t.y = (lin / nx) % ny;
    t.z = lin / (nx * ny);
  } else {
    t.y = lin % ny;
    t.x = (lin / ny) % nx;
    t.z = lin / (nx * ny);
  }
  return t;
}

template <bool TA, bool TB>
__global__ void __launch_bounds__(256)
gemm_k(int M, int N, int K, int kchunk, float alpha, const float* __restrict__ A, long long lda, int veca,
       const float* __restrict__ B, long long ldb, int vecb, float* __restrict__ C, long long ldc, float beta,
       const float* __restrict__ bias, int act, int auxm, const float* __restrict__ aux, long long ldaux,
       float* __restrict__ part, float* __restrict__ rowsum, float* __restrict__ rowpart, PendEpi pe) {
  PAIG_PENDING_EPI(pe)
  __shared__ __attribute__((aligned(16))) float As[IMG];
  __shared__ __attribute__((aligned(16))) float Bs[IMG];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  const TileId bt = xcd_tile((int)gridDim.z - (pe.S ? 1 : 0));
  const int m0 = bt.y * BM, n0 = bt.x * BN;
  const int kbeg = bt.z * kchunk;
  int kend = kbeg + kchunk;
  if (kend > K) kend = K;
  const bool do_rs = rowsum != nullptr && bt.x == 0;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float rs = 0.f;

  Tile<!TA> ta;  // A is k-contiguous unless transposed
  Tile<TB> tb;   // B is k-contiguous when transposed
  if (kbeg < kend) {
    ta.load(A, lda, m0, kbeg, M, kend, veca, tid);
    tb.load(B, ldb, n0, kbeg, N, kend, vecb, tid);
  }
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    __syncthreads();
    ta.store(As, tid);
    tb.store(Bs, tid);
    __syncthreads();
    if (k0 + BK < kend) {   // prefetch the next K tile into registers
      ta.load(A, lda, m0, k0 + BK, M, kend, veca, tid);
      tb.load(B, ldb, n0, k0 + BK, N, kend, vecb, tid);
    }
    if (do_rs && tid < BM) {
#pragma unroll 8
      for (int k = 0; k < BK; ++k) rs += Tile<!TA>::at(As, tid, k);
    }
#pragma unroll
    for (int ks = 0; ks < BK; ks += 4) {
      const int kr = ks + (lane >> 4);
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = Tile<!TA>::at(As, wm * 32 + i * 16 + (lane & 15), kr);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Tile<TB>::at(Bs, wn * 32 + j * 16 + (lane & 15), kr);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
  if (do_rs && tid < BM && m0 + tid < M) {
    if (rowpart) rowpart[(long long)bt.z * M + m0 + tid] = alpha * rs;
    else rowsum[m0 + tid] = alpha * rs;
  }

  // C/D layout: row = (lane>>4)*4 + r, col = lane & 15
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
        const int n = n0 + wn * 32 + j * 16 + (lane & 15);
        if (m < M && n < N) {
          float v = alpha * acc[i][j][r];
          if (part) {
            part[((long long)bt.z * M + m) * N + n] = v;
          } else {
            if (beta != 0.f) v += beta * C[(long long)m * ldc + n];
            if (bias) v += bias[n];
            C[(long long)m * ldc + n] = epi(v, act, auxm, aux, (long long)m * ldaux + n);
          }
        }
      }
}

// ============================================ split-precision 16-bit MFMA GEMM
// The same contract on v_mfma_f32_16x16x32_{f16,bf16}: every fp32 operand is
// split into hi + lo 16-bit parts while it is staged (v = hi + lo exactly up
// to the lo rounding) and a product is hi*hi + hi*lo + lo*hi, fp32 accumulate.
// Per K element the three MFMAs cost ~3/16 of the f32-input form, so these
// GEMMs (K = 3072 / 2000 / 200) fall to the HBM roofline.  math: 1 = f16
// pieces (22 significant bits; operands must satisfy |v| < 65504: forward
// activations / weights, range-guarded, see common.h), 4 = f16 pieces for a
// backward GEMM: op(A) (the gradient, any magnitude) scaled by a running
// block power of two (each K-tile's max |op(A)| into [2^14, 2^15); a tile that
// needs a smaller exponent first rescales the accumulators exactly), op(B)
// (weights, bounded) at the fixed 2^PAIG_A_EXP, range-guarded; 5 = both
// operands at the fixed 2^PAIG_A_EXP, range-guarded; 6 = both operands with
// running exponents (a wgrad GEMM: gradient x activations).  Scaling keeps 22 significant bits for all but negligibly
// small values (an unscaled f16 lo piece is subnormal below |v| = 1/8);
// 2 = bf16 pieces (16 bits, fp32 range; kept for the ABI, not used by the
// step: its gradient errors measured well outside the fp32 envelope), 3 =
// bf16 hi only (the bf16 configuration).
// LDS images keep each operand's global orientation: k-contiguous operands
// as [row][k] (pitch 48, see SPK), row-contiguous operands as [pi(k)][row] (pitch 80) read with
// ds_read_b64_tr_b16; pi places the 8 k-rows one 32-lane half reads in 8
// consecutive image rows, 5 x 32 B apart mod 256 B: conflict-free.
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

// [row][k] pitch (16-bit elements): 6 16-B slots.  ds_read_b128 serves a
// wave in lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32): 8 rows at
// k-offset g and 8 rows at g+1 slot.  A pitch of 2 (mod 4) slots puts the 8
// rows of one on the 8 even slots of a 256-B bank row and the other 8 on the
// odd ones (the former 5-slot pitch collided 2-way)
constexpr int SPK = 48;
constexpr int SPR = 80;          // [pi(k)][row] pitch
constexpr int SIMG = 64 * SPK > BK * SPR ? 64 * SPK : BK * SPR;

__device__ __forceinline__ int kperm(int k) {   // k = 8g + 4h + q
  const int g = k >> 3, h = (k >> 2) & 1, q = k & 3;
  return 16 * (g >> 1) + 8 * h + 4 * (g & 1) + q;
}

// f16-piece modes, and the ones whose operands are scaled by powers of two
#define F16PM(PM) ((PM) == 1 || (PM) == 4 || (PM) == 5 || (PM) == 6)
#define SCALED(PM) ((PM) >= 4)

template <int PM>
__device__ __forceinline__ void gsplit(float v, short& h, short& l, float& rmax) {
  if constexpr (F16PM(PM)) {
    rmax = fmaxf(rmax, fabsf(v));
    const _Float16 a = (_Float16)v;
    h = __builtin_bit_cast(short, a);
    l = __builtin_bit_cast(short, (_Float16)(v - (float)a));
  } else {
    const __bf16 a = (__bf16)v;
    h = __builtin_bit_cast(short, a);
    l = PM == 2 ? __builtin_bit_cast(short, (__bf16)(v - (float)a)) : (short)0;
  }
}

template <int PM>
__device__ __forceinline__ f32x4 gmma(s16x8 a, s16x8 b, f32x4 c) {
  if constexpr (F16PM(PM))
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                  0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
}

// 16-bit image of one 64 x BK operand tile (the fp32 Tile registers times
// sc, split)
template <bool KCONTIG, int PM>
__device__ __forceinline__ void store16(const Tile<KCONTIG>& t, short* ih, short* il, int tid, float sc,
                                        float& rmax) {
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    s16x4 hv, lv;
    if constexpr (F16PM(PM)) {
      // packed multiplies and conversions (split_pk), pairs of consecutive elements
      const pf32x2 a = pf32x2{t.v[e][0], t.v[e][1]} * sc, b = pf32x2{t.v[e][2], t.v[e][3]} * sc;
      rmax = amax2(amax2(rmax, a.x, a.y), b.x, b.y);
      u32x2 h, l;
      { const HiLo q_ = split_pk(a.x, a.y); h[0] = q_.h; l[0] = q_.l; }
      { const HiLo q_ = split_pk(b.x, b.y); h[1] = q_.h; l[1] = q_.l; }
      hv = __builtin_bit_cast(s16x4, h);
      lv = __builtin_bit_cast(s16x4, l);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        short h, l;
        gsplit<PM>(t.v[e][i] * sc, h, l, rmax);
        hv[i] = h;
        lv[i] = l;
      }
    }
    int o;
    if (KCONTIG) o = ((tid >> 3) + 32 * e) * SPK + (tid & 7) * 4;
    else o = kperm((tid >> 4) + 16 * e) * SPR + (tid & 15) * 4;
    *reinterpret_cast<s16x4*>(ih + o) = hv;
    if (PM != 3) *reinterpret_cast<s16x4*>(il + o) = lv;
  }
}

// fragment of 16 rows (r0 ..) x 32 k for this lane: row r0 + (lane & 15), k = 8(lane>>4) + j
template <bool KCONTIG>
__device__ __forceinline__ s16x8 frag16(const short* img, int r0, int lane) {
  if (KCONTIG) return *reinterpret_cast<const s16x8*>(img + (r0 + (lane & 15)) * SPK + 8 * (lane >> 4));
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const short* b0 = img + kperm(8 * g + q) * SPR + r0 + 4 * p;
  const short* b1 = img + kperm(8 * g + 4 + q) * SPR + r0 + 4 * p;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)b0);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)b1);
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// Occupancy over ring depth: the l1 dgrad's 1536 blocks fit the 256 CUs in
// one round at 6 blocks per CU (LDS allows 6), i.e. <= 80 VGPRs; a 3-deep
// register ring needs 124 (4 per CU: two rounds), and 2-deep spills at 80.
// Measured (tools/gemm_bench.py): depth 1 at 6 waves/SIMD 27.6 us vs 31.7 us
// for that GEMM, the others unchanged; the step 1.168 vs 1.177 ms
template <bool TA, bool TB, int PM, bool VEC>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6)))
gemm_split_k(int M, int N, int K, int kchunk, float alpha, const float* __restrict__ A, long long lda, int veca,
             const float* __restrict__ B, long long ldb, int vecb, float* __restrict__ C, long long ldc, float beta,
             const float* __restrict__ bias, int act, int auxm, const float* __restrict__ aux, long long ldaux,
             float* __restrict__ part, float* __restrict__ rowsum, float* __restrict__ rowpart, PendEpi pe) {
  PAIG_PENDING_EPI(pe)
  constexpr int NI = PM == 3 ? 1 : 2;
  __shared__ __attribute__((aligned(16))) short S16[4 * SIMG];
  short* Ah = S16;
  short* Al = S16 + SIMG;
  short* Bh = S16 + 2 * SIMG;
  short* Bl = S16 + 3 * SIMG;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  const TileId bt = xcd_tile((int)gridDim.z - (pe.S ? 1 : 0));
  const int m0 = bt.y * BM, n0 = bt.x * BN;
  const int kbeg = bt.z * kchunk;
  int kend = kbeg + kchunk;
  if (kend > K) kend = K;
  // row sums of op(A) (= the bias gradient of a wgrad GEMM) in exact fp32
  // from the staging registers; only the transposed-A form carries them
  const bool do_rs = TA && rowsum != nullptr && bt.x == 0;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 rs4 = f32x4{0.f, 0.f, 0.f, 0.f};
  float rmax = 0.f;                                   // f16 range guard of fixed-scale operands
  // operand scales 2^eca, 2^ecb: dynamic ones (DA: PM 4, 6; DB: PM 6) run
  // from a high start down to each K-tile's need; the fixed ones (PM 5: both,
  // PM 4: op(B)) are the activation / weight scale 2^PAIG_A_EXP
  constexpr bool DA = PM == 4 || PM == 6, DB = PM == 6;
  int eca = DA ? 100 : (PM == 5 ? PAIG_A_EXP : 0);
  int ecb = DB ? 100 : (PM == 4 || PM == 5 ? PAIG_A_EXP : 0);
  float asc = __builtin_amdgcn_ldexpf(1.f, eca);
  float bsc = __builtin_amdgcn_ldexpf(1.f, ecb);
  __shared__ float smx[8];

  // register ring of NS K-tiles: the loads of tile k + NS are issued right
  // after tile k is parked in LDS, so they fly behind tile k's MFMAs (and
  // the other 5 blocks of the CU hide the rest; see the occupancy note above)
  constexpr int NS = 1;
  Tile<!TA> ta[NS];
  Tile<TB> tb[NS];
#pragma unroll
  for (int st = 0; st < NS; ++st) {   // (tiles past kend load as zeros)
    ta[st].template load_bf<VEC>(A, lda, m0, kbeg + st * BK, M, kend, tid);
    tb[st].template load_bf<VEC>(B, ldb, n0, kbeg + st * BK, N, kend, tid);
  }
  for (int k0 = kbeg; k0 < kend; k0 += NS * BK) {
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      const int kk = k0 + st * BK;
      // a stage past kend skips its work (uniform branch) but still issues
      // its (zero) ring loads: every path then issues the same loads in the
      // same order, so the compiler's wait before a stage's use counts the
      // NS-1 tiles behind it (a `break` here made it drain the whole ring at
      // the top of every NS-tile group)
      if (kk < kend) {
      // this K-tile's max |op(A)| / |op(B)| (dynamic operands), published
      // before the barrier (the previous tile's smx reads finished before the
      // last one)
      if constexpr (DA) {
        float ma = 0.f;
#pragma unroll
        for (int e = 0; e < 2; ++e) ma = amax2(amax2(ma, ta[st].v[e][0], ta[st].v[e][1]), ta[st].v[e][2], ta[st].v[e][3]);
        ma = wave_max_u(ma);
        if (lane == 0) smx[wv] = ma;
      }
      if constexpr (DB) {
        float mb = 0.f;
#pragma unroll
        for (int e = 0; e < 2; ++e) mb = amax2(amax2(mb, tb[st].v[e][0], tb[st].v[e][1]), tb[st].v[e][2], tb[st].v[e][3]);
        mb = wave_max_u(mb);
        if (lane == 0) smx[4 + wv] = mb;
      }
      __syncthreads();
      if constexpr (DA || DB) {
        // a smaller exponent than the running one rescales the accumulators
        // (held at 2^(eca + ecb)) exactly first
        int na = eca, nb = ecb;
        if constexpr (DA) na = min(eca, f16_scale_exp(fmaxf(fmaxf(smx[0], smx[1]), fmaxf(smx[2], smx[3]))));
        if constexpr (DB) nb = min(ecb, f16_scale_exp(fmaxf(fmaxf(smx[4], smx[5]), fmaxf(smx[6], smx[7]))));
        if (na + nb < eca + ecb) {
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                acc[i][j][r] = __builtin_amdgcn_ldexpf(acc[i][j][r], (na + nb) - (eca + ecb));
        }
        eca = na;
        ecb = nb;
        asc = __builtin_amdgcn_ldexpf(1.f, eca);
        bsc = __builtin_amdgcn_ldexpf(1.f, ecb);
      }
      float dmx = 0.f;   // dynamically scaled operands stay below 2^15: no guard
      store16<!TA, PM>(ta[st], Ah, Al, tid, asc, DA ? dmx : rmax);
      store16<TB, PM>(tb[st], Bh, Bl, tid, bsc, DB ? dmx : rmax);
      if (do_rs) rs4 += ta[st].v[0] + ta[st].v[1];
      __syncthreads();
      }
      ta[st].template load_bf<VEC>(A, lda, m0, kk + NS * BK, M, kend, tid);
      tb[st].template load_bf<VEC>(B, ldb, n0, kk + NS * BK, N, kend, tid);
      if (kk < kend) {
      s16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        ah[i] = frag16<!TA>(Ah, wm * 32 + i * 16, lane);
        al[i] = PM != 3 ? frag16<!TA>(Al, wm * 32 + i * 16, lane) : ah[i];
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        bh[j] = frag16<TB>(Bh, wn * 32 + j * 16, lane);
        bl[j] = PM != 3 ? frag16<TB>(Bl, wn * 32 + j * 16, lane) : bh[j];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if constexpr (PM != 3) {
            acc[i][j] = gmma<PM>(al[i], bh[j], acc[i][j]);
            acc[i][j] = gmma<PM>(ah[i], bl[j], acc[i][j]);
          }
          acc[i][j] = gmma<PM>(ah[i], bh[j], acc[i][j]);
        }
      }
    }
  }
  if (do_rs) {
    // thread (k = tid>>4 (+16), rows (tid&15)*4 .. +3): reduce over the 16 k-threads
    __syncthreads();
    float* red = reinterpret_cast<float*>(S16);   // [16][64]
    *reinterpret_cast<f32x4*>(red + (tid >> 4) * 64 + (tid & 15) * 4) = rs4;
    __syncthreads();
    if (tid < BM && m0 + tid < M) {
      float v = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) v += red[k * 64 + tid];
      if (rowpart) rowpart[(long long)bt.z * M + m0 + tid] = alpha * v;
      else rowsum[m0 + tid] = alpha * v;
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
        const int n = n0 + wn * 32 + j * 16 + (lane & 15);
        if (m < M && n < N) {
          float v = alpha * (SCALED(PM) ? __builtin_amdgcn_ldexpf(acc[i][j][r], -(eca + ecb)) : acc[i][j][r]);
          if (part) {
            part[((long long)bt.z * M + m) * N + n] = v;
          } else {
            if (beta != 0.f) v += beta * C[(long long)m * ldc + n];
            if (bias) v += bias[n];
            C[(long long)m * ldc + n] = epi(v, act, auxm, aux, (long long)m * ldaux + n);
          }
        }
      }
  if constexpr (F16PM(PM)) f16_range_note(rmax);
}

// ------------------------------------------------- wide tiles (512 threads)
// The same split-precision contract on 64 x 256 or 256 x 64 block tiles, for
// the encoder projection's shapes (l1: 2000 x 200 x 3072 forward, 200 x 3072
// x 2000 wgrad, 2000 x 3072 x 200 dgrad): one block spans the whole narrow
// dimension (<= 256), so the wide operand is loaded, scaled and split ONCE
// instead of once per 64-column tile (the 64 x 64 form converts the 24.6 MB
// activation operand 4x and re-reads it from L2 4x), and each wave's K step
// carries 2-3x the MFMAs per fragment read and barrier.  8 waves as WM x WN,
// each a (BMT/WM) x (BNT/WN) patch of 16 x 16 MFMA tiles.
template <bool KCONTIG, int ROWS>
struct WTile {
  static constexpr int NTHR = 512;
  static constexpr int E = ROWS * BK / (4 * NTHR);   // float4 per thread: 64 rows -> 1, 256 -> 4
  static constexpr int RQ = ROWS / 4;                // !KCONTIG: float4 per k-row
  f32x4 v[E];
  static __device__ __forceinline__ void rk(int tid, int e, int& r, int& k) {
    if (KCONTIG) { r = (tid >> 3) + (NTHR / 8) * e; k = (tid & 7) * 4; }
    else { r = (tid % RQ) * 4; k = tid / RQ + (NTHR / RQ) * e; }
  }
  template <bool VEC>
  __device__ __forceinline__ void load_bf(const float* __restrict__ p, long long ld, int r0, int k0, int R, int K,
                                          int tid) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      int r, k;
      rk(tid, e, r, k);
      const int gr = r0 + r, gk = k0 + k;
      if constexpr (VEC) {
        const bool ok = gr < R && gk < K;
        const float* q = ok ? p + (KCONTIG ? (long long)gr * ld + gk : (long long)gk * ld + gr) : zero16;
        v[e] = *reinterpret_cast<const f32x4*>(q);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rr = KCONTIG ? gr : gr + i, kk = KCONTIG ? gk + i : gk;
          const bool ok = rr < R && kk < K;
          v[e][i] = *(ok ? p + (KCONTIG ? (long long)rr * ld + kk : (long long)kk * ld + rr) : zero16);
        }
      }
    }
  }
  // [pi(k)][row] pitch: ROWS + 16 shorts = an odd multiple of 32 B, so the
  // 8 image rows a half-wave's ds_read_b64_tr_b16 reads hit 8 distinct 32-B
  // bank groups (64 rows: 160 B, 256 rows: 544 B = 32 mod 256)
  static constexpr int SPRW = ROWS + 16;
  static constexpr int IMG = ROWS * SPK > BK * SPRW ? ROWS * SPK : BK * SPRW;
  template <int PM>
  __device__ __forceinline__ void store16(short* ih, short* il, int tid, float sc, float& rmax) const {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const pf32x2 a = pf32x2{v[e][0], v[e][1]} * sc, b = pf32x2{v[e][2], v[e][3]} * sc;
      s16x4 hv, lv;
      if constexpr (F16PM(PM)) {
        rmax = amax2(amax2(rmax, a.x, a.y), b.x, b.y);
        u32x2 h, l;
        { const HiLo q_ = split_pk(a.x, a.y); h[0] = q_.h; l[0] = q_.l; }
        { const HiLo q_ = split_pk(b.x, b.y); h[1] = q_.h; l[1] = q_.l; }
        hv = __builtin_bit_cast(s16x4, h);
        lv = __builtin_bit_cast(s16x4, l);
      } else {
        const float t[4] = {a.x, a.y, b.x, b.y};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          short hh, ll;
          gsplit<PM>(t[i], hh, ll, rmax);
          hv[i] = hh;
          lv[i] = ll;
        }
      }
      int r, k;
      rk(tid, e, r, k);
      const int o = KCONTIG ? r * SPK + k : kperm(k) * SPRW + r;
      *reinterpret_cast<s16x4*>(ih + o) = hv;
      if (PM != 3) *reinterpret_cast<s16x4*>(il + o) = lv;
    }
  }
  __device__ __forceinline__ float amax() const {
    float m = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) m = amax2(amax2(m, v[e][0], v[e][1]), v[e][2], v[e][3]);
    return m;
  }
  static __device__ __forceinline__ s16x8 frag(const short* img, int r0, int lane) {
    if (KCONTIG) return *reinterpret_cast<const s16x8*>(img + (r0 + (lane & 15)) * SPK + 8 * (lane >> 4));
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const short* b0 = img + kperm(8 * g + q) * SPRW + r0 + 4 * p;
    const short* b1 = img + kperm(8 * g + 4 + q) * SPRW + r0 + 4 * p;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)b0);
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)b1);
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  }
};

template <bool TA, bool TB, int PM, bool VEC, int BMT, int BNT>
__global__ void __launch_bounds__(512)
gemm_split_w_k(int M, int N, int K, int kchunk, float alpha, const float* __restrict__ A, long long lda, int veca,
               const float* __restrict__ B, long long ldb, int vecb, float* __restrict__ C, long long ldc, float beta,
               const float* __restrict__ bias, int act, int auxm, const float* __restrict__ aux, long long ldaux,
               float* __restrict__ part, float* __restrict__ rowsum, float* __restrict__ rowpart, PendEpi pe) {
  PAIG_PENDING_EPI(pe)
  constexpr int WM = BMT == 64 ? 2 : 4, WN = 8 / WM;
  constexpr int PMW = BMT / WM, PNW = BNT / WN;          // wave patch
  constexpr int MI = PMW / 16, NJ = PNW / 16;
  using TTA = WTile<!TA, BMT>;
  using TTB = WTile<TB, BNT>;
  constexpr int IA = TTA::IMG, IB = TTB::IMG;
  __shared__ __attribute__((aligned(16))) short S16[2 * IA + 2 * IB];
  short* Ah = S16;
  short* Al = S16 + IA;
  short* Bh = S16 + 2 * IA;
  short* Bl = Bh + IB;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const int wm = wv / WN, wn = wv % WN;
  const TileId bt = xcd_tile((int)gridDim.z - (pe.S ? 1 : 0));
  const int m0 = bt.y * BMT, n0 = bt.x * BNT;
  const int kbeg = bt.z * kchunk;
  int kend = kbeg + kchunk;
  if (kend > K) kend = K;
  const bool do_rs = TA && rowsum != nullptr && bt.x == 0;

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 rs4 = f32x4{0.f, 0.f, 0.f, 0.f};
  float rmax = 0.f;
  constexpr bool DA = PM == 4 || PM == 6, DB = PM == 6;
  int eca = DA ? 100 : (PM == 5 ? PAIG_A_EXP : 0);
  int ecb = DB ? 100 : (PM == 4 || PM == 5 ? PAIG_A_EXP : 0);
  float asc = __builtin_amdgcn_ldexpf(1.f, eca);
  float bsc = __builtin_amdgcn_ldexpf(1.f, ecb);
  __shared__ float smx[16];

  constexpr int NS = 3;
  TTA ta[NS];
  TTB tb[NS];
#pragma unroll
  for (int st = 0; st < NS; ++st) {
    ta[st].template load_bf<VEC>(A, lda, m0, kbeg + st * BK, M, kend, tid);
    tb[st].template load_bf<VEC>(B, ldb, n0, kbeg + st * BK, N, kend, tid);
  }
  for (int k0 = kbeg; k0 < kend; k0 += NS * BK) {
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      const int kk = k0 + st * BK;
      if (kk < kend) {   // (no break: see gemm_split_k)
      if constexpr (DA) {
        const float ma = wave_max_u(ta[st].amax());
        if (lane == 0) smx[wv] = ma;
      }
      if constexpr (DB) {
        const float mb = wave_max_u(tb[st].amax());
        if (lane == 0) smx[8 + wv] = mb;
      }
      __syncthreads();
      if constexpr (DA || DB) {
        int na = eca, nb = ecb;
        if constexpr (DA) {
          float m = smx[0];
#pragma unroll
          for (int w = 1; w < 8; ++w) m = fmaxf(m, smx[w]);
          na = min(eca, f16_scale_exp(m));
        }
        if constexpr (DB) {
          float m = smx[8];
#pragma unroll
          for (int w = 9; w < 16; ++w) m = fmaxf(m, smx[w]);
          nb = min(ecb, f16_scale_exp(m));
        }
        if (na + nb < eca + ecb) {
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                acc[i][j][r] = __builtin_amdgcn_ldexpf(acc[i][j][r], (na + nb) - (eca + ecb));
        }
        eca = na;
        ecb = nb;
        asc = __builtin_amdgcn_ldexpf(1.f, eca);
        bsc = __builtin_amdgcn_ldexpf(1.f, ecb);
      }
      float dmx = 0.f;
      ta[st].template store16<PM>(Ah, Al, tid, asc, DA ? dmx : rmax);
      tb[st].template store16<PM>(Bh, Bl, tid, bsc, DB ? dmx : rmax);
      if (do_rs) {
#pragma unroll
        for (int e = 0; e < TTA::E; ++e) rs4 += ta[st].v[e];
      }
      __syncthreads();
      }
      ta[st].template load_bf<VEC>(A, lda, m0, kk + NS * BK, M, kend, tid);
      tb[st].template load_bf<VEC>(B, ldb, n0, kk + NS * BK, N, kend, tid);
      if (kk < kend) {
      s16x8 ah[MI], al[MI], bh[NJ], bl[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        ah[i] = TTA::frag(Ah, wm * PMW + i * 16, lane);
        al[i] = PM != 3 ? TTA::frag(Al, wm * PMW + i * 16, lane) : ah[i];
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        bh[j] = TTB::frag(Bh, wn * PNW + j * 16, lane);
        bl[j] = PM != 3 ? TTB::frag(Bl, wn * PNW + j * 16, lane) : bh[j];
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          if constexpr (PM != 3) {
            acc[i][j] = gmma<PM>(al[i], bh[j], acc[i][j]);
            acc[i][j] = gmma<PM>(ah[i], bl[j], acc[i][j]);
          }
          acc[i][j] = gmma<PM>(ah[i], bh[j], acc[i][j]);
        }
      }
    }
  }
  if (do_rs) {
    // op(A) = A^T is the !KCONTIG tile: thread rows (tid % RQ)*4 .. +3; the
    // NTHR / RQ threads of one row group are combined in a fixed order
    constexpr int RQ = TTA::RQ, G = 512 / RQ;
    __syncthreads();
    float* red = reinterpret_cast<float*>(S16);   // [G][BMT]
    *reinterpret_cast<f32x4*>(red + (tid / RQ) * BMT + (tid % RQ) * 4) = rs4;
    __syncthreads();
    if (tid < BMT && m0 + tid < M) {
      float v = 0.f;
#pragma unroll
      for (int k = 0; k < G; ++k) v += red[k * BMT + tid];
      if (rowpart) rowpart[(long long)bt.z * M + m0 + tid] = alpha * v;
      else rowsum[m0 + tid] = alpha * v;
    }
  }
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * PMW + i * 16 + (lane >> 4) * 4 + r;
        const int n = n0 + wn * PNW + j * 16 + (lane & 15);
        if (m < M && n < N) {
          float v = alpha * (SCALED(PM) ? __builtin_amdgcn_ldexpf(acc[i][j][r], -(eca + ecb)) : acc[i][j][r]);
          if (part) {
            part[((long long)bt.z * M + m) * N + n] = v;
          } else {
            if (beta != 0.f) v += beta * C[(long long)m * ldc + n];
            if (bias) v += bias[n];
            C[(long long)m * ldc + n] = epi(v, act, auxm, aux, (long long)m * ldaux + n);
          }
        }
      }
  if constexpr (F16PM(PM)) f16_range_note(rmax);
}

// sum_{s<S} p[s*ld] in order s = 0..S-1 (deterministic), loads issued 8 at a
// time so the partial slabs stream instead of one dependent load per split
__device__ __forceinline__ float sum_strided(const float* __restrict__ p, long long ld, int S) {
  float v = 0.f;
  int s = 0;
  for (; s + 8 <= S; s += 8) {
    float t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = p[(long long)(s + j) * ld];
#pragma unroll
    for (int j = 0; j < 8; ++j) v += t[j];
  }
  for (; s < S; ++s) v += p[(long long)s * ld];
  return v;
}

__device__ __forceinline__ void splitk_epi_scalar(int M, int N, int S, const float* __restrict__ part,
                                                  float* __restrict__ C, long long ldc, float beta,
                                                  const float* __restrict__ bias, int act, int auxm,
                                                  const float* __restrict__ aux, long long ldaux,
                                                  const float* __restrict__ rowpart, float* __restrict__ rowsum, int bid,
                                                  int nb) {
  const long long n_el = (long long)M * N;
  const long long tot = n_el + (rowsum ? M : 0);
  for (long long i = bid * (long long)blockDim.x + threadIdx.x; i < tot; i += (long long)nb * blockDim.x) {
    if (i >= n_el) {
      const int m = (int)(i - n_el);
      rowsum[m] = sum_strided(rowpart + m, M, S);
      continue;
    }
    const int m = (int)(i / N), n = (int)(i % N);
    float v = sum_strided(part + i, n_el, S);
    if (beta != 0.f) v += beta * C[(long long)m * ldc + n];
    if (bias) v += bias[n];
    C[(long long)m * ldc + n] = epi(v, act, auxm, aux, (long long)m * ldaux + n);
  }
}
__global__ void gemm_splitk_epilogue_k(int M, int N, int S, const float* __restrict__ part, float* __restrict__ C,
                                       long long ldc, float beta, const float* __restrict__ bias, int act, int auxm,
                                       const float* __restrict__ aux, long long ldaux, const float* __restrict__ rowpart,
                                       float* __restrict__ rowsum) {
  splitk_epi_scalar(M, N, S, part, C, ldc, beta, bias, act, auxm, aux, ldaux, rowpart, rowsum, blockIdx.x, gridDim.x);
}

// Vector form (N % 4 == 0; C, bias, aux and the slabs float4-addressable;
// S * M * N < 2^31; M * N >= 2^19 so the grid stays wide): 4 consecutive
// columns per thread, float4 loads of up to 8 partials in flight, 32-bit indexing.  The row sums, if any, take the
// threads past the element range.  Same per-element order as the scalar form.
__device__ __forceinline__ void splitk_epi_vec(int M, int N, int S, const float* __restrict__ part,
                                               float* __restrict__ C, int ldc, float beta,
                                               const float* __restrict__ bias, int act, int auxm,
                                               const float* __restrict__ aux, int ldaux,
                                               const float* __restrict__ rowpart, float* __restrict__ rowsum, int bid,
                                               int nb) {
  const int n_el = M * N, n4 = n_el >> 2;
  const int tot = n4 + (rowsum ? M : 0);
  for (int i = bid * blockDim.x + threadIdx.x; i < tot; i += nb * blockDim.x) {
    if (i >= n4) {
      const int m = i - n4;
      rowsum[m] = sum_strided(rowpart + m, M, S);
      continue;
    }
    const int e = i << 2, m = e / N, n = e - m * N;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    int s = 0;
    for (; s + 8 <= S; s += 8) {   // 8 partial loads in flight, summed in slab order
      float4 t[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = *reinterpret_cast<const float4*>(part + (s + j) * n_el + e);
#pragma unroll
      for (int j = 0; j < 8; ++j) { v.x += t[j].x; v.y += t[j].y; v.z += t[j].z; v.w += t[j].w; }
    }
    for (; s < S; ++s) {
      const float4 a = *reinterpret_cast<const float4*>(part + s * n_el + e);
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    }
    float* c = C + m * ldc + n;
    if (beta != 0.f) {
      const float4 o = *reinterpret_cast<const float4*>(c);
      v.x += beta * o.x; v.y += beta * o.y; v.z += beta * o.z; v.w += beta * o.w;
    }
    if (bias) {
      const float4 b = *reinterpret_cast<const float4*>(bias + n);
      v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
    }
    const long long ao = (long long)m * ldaux + n;
    v.x = epi(v.x, act, auxm, aux, ao);
    v.y = epi(v.y, act, auxm, aux, ao + 1);
    v.z = epi(v.z, act, auxm, aux, ao + 2);
    v.w = epi(v.w, act, auxm, aux, ao + 3);
    *reinterpret_cast<float4*>(c) = v;
  }
}
__global__ void __launch_bounds__(256) gemm_splitk_epilogue_v_k(int M, int N, int S, const float* __restrict__ part,
                                                                float* __restrict__ C, int ldc, float beta,
                                                                const float* __restrict__ bias, int act, int auxm,
                                                                const float* __restrict__ aux, int ldaux,
                                                                const float* __restrict__ rowpart,
                                                                float* __restrict__ rowsum) {
  splitk_epi_vec(M, N, S, part, C, ldc, beta, bias, act, auxm, aux, ldaux, rowpart, rowsum, blockIdx.x, gridDim.x);
}

__device__ void splitk_epi_run(const PendEpi& pe, int bid, int nb) {
  if (pe.v4)
    splitk_epi_vec(pe.M, pe.N, pe.S, pe.part, pe.C, (int)pe.ldc, pe.beta, pe.bias, pe.act, pe.auxm, pe.aux,
                   (int)pe.ldaux, pe.rowpart, pe.rowsum, bid, nb);
  else
    splitk_epi_scalar(pe.M, pe.N, pe.S, pe.part, pe.C, pe.ldc, pe.beta, pe.bias, pe.act, pe.auxm, pe.aux, pe.ldaux,
                      pe.rowpart, pe.rowsum, bid, nb);
}

// Split-K factor: the dense layers here are small (M, N <= a few thousand)
// and latency-bound, so split until ~2 blocks per CU are in flight (measured
// best: 4 per CU paid more in partial-slab traffic than it won), keeping
// >= 1 BK step per split and the partial slabs <= 16 MB.
static int choose_split(int M, int N, int K) {
  const int tiles = cdiv(M, BM) * cdiv(N, BN);
  int s = 1;
  if (K < 512) {
    // a short K loop usually costs less than the split-K epilogue launch;
    // A/B (PAIG_GEMM_SMALLK=1): halve K when the grid fills < 256 CUs.  The
    // split then depends on K and the tile count, never on the row order.
    static int sk = -1;
    if (sk < 0) {
      const char* e = getenv("PAIG_GEMM_SMALLK");
      sk = e ? atoi(e) : 0;
    }
    return (sk && tiles < 256 && K >= 4 * BK) ? 2 : 1;
  }
  while (tiles * s < 512 && cdiv(K, 2 * s) >= BK && (long long)(2 * s) * M * N <= (4ll << 20)) s *= 2;
  return s;
}

// Tile plan: 0 = 64 x 64 (256 threads), 1 = 64 x 256, 2 = 256 x 64 (wide,
// 512 threads, split-precision maths only).  A wide tile spans a narrow
// dimension of 129..256 whole, when the grid still has >= 128 blocks.
// PAIG_GEMM_TILE=0 in the environment forces the 64 x 64 form (A/B runs).
struct GemmPlan {
  int tile, S;
};
static int gemm_tile_env() {
  static int v = -2;
  if (v == -2) {
    const char* e = getenv("PAIG_GEMM_TILE");
    v = e ? atoi(e) : -1;
  }
  return v;
}
static GemmPlan plan_gemm(int M, int N, int K, int math) {
  GemmPlan p{0, K > 0 ? choose_split(M, N, K) : 1};
  if (!(math == 3 || math == 4 || math == 6) || gemm_tile_env() == 0 || K <= 0) return p;
  // measured (tools/gemm_bench.py): the 64 x 256 tile wins where it holds the
  // whole N and K is split (the projection forward, 34.8 -> 28.6 us); the
  // l1 dgrad (N = 3072, K = 200) and the 256 x 64 wgrad tile fill fewer CUs
  // and lost 20% each, so they keep the 64 x 64 form
  int tile = 0;
  if (N > 128 && N <= 256 && M >= 512 && K >= 512) tile = 1;
  if (!tile) return p;
  // the split depends on K alone (~12 K-steps per block), so a row's sum
  // order does not change with M: a half batch reproduces the full batch's
  // rows exactly (the data-parallel AVG identity, tests/test_gpu_fullsize.py)
  int S = 1;
  while (K / (2 * S) >= 384) S *= 2;
  if ((long long)S * M * N > (8ll << 20) || cdiv(M, 64) * S < 128) return p;
  return GemmPlan{tile, S};
}

static inline bool vec_ok(const float* p, long long ld) {
  return ((uintptr_t)p % 16 == 0) && (ld % 4 == 0);
}

template <bool TA, bool TB>
static void launch_gemm(int math, int tile, dim3 grid, hipStream_t st, int M, int N, int K, int kchunk, float alpha,
                        const float* A, long long lda, int va, const float* B, long long ldb, int vb, float* C,
                        long long ldc, float beta, const float* bias, int act, int auxm, const float* aux,
                        long long ldaux, float* part, float* rowsum, float* rowpart, const PendEpi& pe) {
  if (pe.S) grid.z += 1;   // the deferred epilogue's plane
#define PAIG_L(KERN)                                                                                          \
  hipLaunchKernelGGL(KERN, grid, dim3(256), 0, st, M, N, K, kchunk, alpha, A, lda, va, B, ldb, vb, C, ldc, beta, \
                     bias, act, auxm, aux, ldaux, part, rowsum, rowpart, pe)
  // the split kernels' branch-free loads: float4 when both operands allow
  const bool v = va && vb;
#define PAIG_W(KERN) \
  hipLaunchKernelGGL(KERN, grid, dim3(512), 0, st, M, N, K, kchunk, alpha, A, lda, va, B, ldb, vb, C, ldc, beta, \
                     bias, act, auxm, aux, ldaux, part, rowsum, rowpart, pe)
#define PAIG_S(PM_) \
  do {                                              \
    if (v) PAIG_L((gemm_split_k<TA, TB, PM_, true>)); \
    else PAIG_L((gemm_split_k<TA, TB, PM_, false>));  \
  } while (0)
  // wide tiles: the step's maths (3, 4, 6) with float4 operands (plan_gemm)
#define PAIG_SW(PM_) \
  do {                                                                  \
    if (tile == 1) PAIG_W((gemm_split_w_k<TA, TB, PM_, true, 64, 256>)); \
    else if (tile == 2) PAIG_W((gemm_split_w_k<TA, TB, PM_, true, 256, 64>)); \
    else PAIG_S(PM_);                                                   \
  } while (0)
  if (math == 1) PAIG_S(1);
  else if (math == 2) PAIG_S(2);
  else if (math == 3) PAIG_SW(3);
  else if (math == 4) PAIG_SW(4);
  else if (math == 5) PAIG_S(5);
  else if (math == 6) PAIG_SW(6);
  else PAIG_L((gemm_k<TA, TB>));
#undef PAIG_SW
#undef PAIG_S
#undef PAIG_W
#undef PAIG_L
}

}  // namespace

// split-K epilogue: C = sum_s part[s] (+ beta C) (+ bias) -> act -> * aux'
// (and rowsum = sum_s rowpart[s]); the vector form where the shapes allow
static PendEpi make_epi(int M, int N, int S, const float* part, float* C, long long ldc, float beta, const float* bias,
                        int act, int auxm, const float* aux, long long ldaux, const float* rowpart, float* rowsum) {
  const bool v4 = N % 4 == 0 && vec_ok(C, ldc) && (!bias || (uintptr_t)bias % 16 == 0) &&
                  (!aux || auxm == AUX_NONE || vec_ok(aux, ldaux)) && (uintptr_t)part % 16 == 0 &&
                  (long long)S * M * N < (1ll << 31) && (long long)M * ldc < (1ll << 31) &&
                  (long long)M * ldaux < (1ll << 31) &&
                  (long long)M * N >= (1 << 19);   // smaller outputs keep the scalar form (4x the threads)
  return PendEpi{M, N, S, part, C, ldc, beta, bias, act, auxm, aux, ldaux, rowpart, rowsum, v4 ? 1 : 0};
}
static void launch_epi(const PendEpi& e, hipStream_t st) {
  long long n_el = (e.v4 ? (long long)e.M * e.N / 4 : (long long)e.M * e.N) + (e.rowsum ? e.M : 0);
  int g = cdiv(n_el, 256);
  if (g > 4096) g = 4096;
  if (e.v4)
    hipLaunchKernelGGL(gemm_splitk_epilogue_v_k, dim3(g), dim3(256), 0, st, e.M, e.N, e.S, e.part, e.C, (int)e.ldc,
                       e.beta, e.bias, e.act, e.auxm, e.aux, (int)e.ldaux, e.rowpart, e.rowsum);
  else
    hipLaunchKernelGGL(gemm_splitk_epilogue_k, dim3(g), dim3(256), 0, st, e.M, e.N, e.S, e.part, e.C, e.ldc, e.beta,
                       e.bias, e.act, e.auxm, e.aux, e.ldaux, e.rowpart, e.rowsum);
}
void paig_gemm_splitk_finish(int M, int N, int S, const float* part, float* C, long long ldc, float beta,
                             const float* bias, int act, int auxm, const float* aux, long long ldaux,
                             const float* rowpart, float* rowsum, hipStream_t st) {
  launch_epi(make_epi(M, N, S, part, C, ldc, beta, bias, act, auxm, aux, ldaux, rowpart, rowsum), st);
}

// the deferred epilogue (paig_gemm_defer_epilogue) and the one-shot request
static PendEpi g_pend{};
static bool g_defer_next = false;
static PendEpi take_pending() {
  const PendEpi e = g_pend;
  g_pend = PendEpi{};
  return e;
}

extern "C" {

int paig_gemm_ex(int ta, int tb, int M, int N, int K, float alpha, const float* A, long long lda, const float* B,
                 long long ldb, float beta, float* C, long long ldc, const float* bias, int act, int auxm,
                 const float* aux, long long ldaux, float* rowsum, float* ws, size_t ws_floats, int math,
                 void* stream);

size_t paig_gemm_workspace(int M, int N, int K) {
  // the larger of the two plans (fp32 math always takes the 64 x 64 tiles)
  size_t need = 0;
  for (int math : {0, 4}) {   // 64 x 64 plan, wide plan
    const GemmPlan p = plan_gemm(M, N, K, math);
    if (p.S > 1) need = std::max(need, (size_t)p.S * M * N + (size_t)p.S * M);
  }
  return need;
}

// the next paig_gemm_ex's split-K epilogue waits for the paig_gemm_ex after
// it, whose launch runs it in one more z-plane of blocks (one-shot)
int paig_gemm_defer_epilogue(int on) {
  g_defer_next = on != 0;
  return 0;
}

int paig_gemm_flush(void* stream) {
  const PendEpi e = take_pending();
  if (!e.S) return 0;
  launch_epi(e, (hipStream_t)stream);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_gemm(int ta, int tb, int M, int N, int K, float alpha, const float* A, long long lda, const float* B,
              long long ldb, float beta, float* C, long long ldc, const float* bias, int act, int auxm,
              const float* aux, long long ldaux, float* rowsum, float* ws, size_t ws_floats, void* stream) {
  return paig_gemm_ex(ta, tb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, bias, act, auxm, aux, ldaux, rowsum, ws,
                      ws_floats, 0, stream);
}

size_t paig_gemm_parts_size(int M, int N, int K, int math) {
  if (M <= 0 || N <= 0) return 0;
  const GemmPlan p = plan_gemm(M, N, K, math);
  return (size_t)(p.S > 1 ? p.S : 1) * M * N;
}

int paig_gemm_parts(int ta, int tb, int M, int N, int K, const float* A, long long lda, const float* B,
                    long long ldb, float* part, size_t part_floats, int math, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (int rc = paig_gemm_flush(stream)) return rc;   // (a deferred epilogue runs first)
  PAIG_REQUIRE(math >= 0 && math <= 6, "paig_gemm_parts: math must be 0..6, got %d", math);
  PAIG_REQUIRE(M > 0 && N > 0 && K > 0 && part, "paig_gemm_parts: empty shape (%d x %d x %d) or no slabs", M, N, K);
  const int va = vec_ok(A, lda) && (ta ? M % 4 == 0 : K % 4 == 0);
  const int vb = vec_ok(B, ldb) && (tb ? K % 4 == 0 : N % 4 == 0);
  GemmPlan plan = plan_gemm(M, N, K, math);
  if (plan.tile && !(va && vb)) plan = GemmPlan{0, choose_split(M, N, K)};
  int S = plan.S;
  if (S > 1 && part_floats < (size_t)S * M * N) S = 1;
  PAIG_REQUIRE(part_floats >= (size_t)M * N, "paig_gemm_parts: %zu floats for a %d x %d slab", part_floats, M, N);
  const int kchunk = S > 1 ? cdiv(cdiv(K, S), BK) * BK : K;
  S = cdiv(K, kchunk);
  const int bm = plan.tile == 2 ? 256 : BM, bn = plan.tile == 1 ? 256 : BN;
  dim3 grid(cdiv(N, bn), cdiv(M, bm), S);
#define PAIG_G(TA_, TB_)                                                                                        \
  launch_gemm<TA_, TB_>(math, plan.tile, grid, st, M, N, K, kchunk, 1.f, A, lda, va, B, ldb, vb, nullptr, N, 0.f, \
                        nullptr, 0, 0, nullptr, 0, part, nullptr, nullptr, PendEpi{})
  if (ta && tb) PAIG_G(true, true);
  else if (ta) PAIG_G(true, false);
  else if (tb) PAIG_G(false, true);
  else PAIG_G(false, false);
#undef PAIG_G
  PAIG_CHECK_LAUNCH();
  return S;
}

int paig_gemm_ex(int ta, int tb, int M, int N, int K, float alpha, const float* A, long long lda, const float* B,
                 long long ldb, float beta, float* C, long long ldc, const float* bias, int act, int auxm,
                 const float* aux, long long ldaux, float* rowsum, float* ws, size_t ws_floats, int math,
                 void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (math < 0 || math > 6) {
    paig_set_error("paig_gemm_ex: math must be 0..6, got %d", math);
    return PAIG_E_UNSUPPORTED;
  }
  if (rowsum && !ta) math = 0;   // fused row sums exist on the split path for op(A) = A^T only
  const bool defer = g_defer_next;
  g_defer_next = false;
  if (M <= 0 || N <= 0) return paig_gemm_flush(stream);
  // float4 operand loads: aligned rows and a contiguous extent that is a
  // multiple of 4 (op(A) is k-contiguous unless ta, op(B) when tb)
  const int va = vec_ok(A, lda) && (ta ? M % 4 == 0 : K % 4 == 0);
  const int vb = vec_ok(B, ldb) && (tb ? K % 4 == 0 : N % 4 == 0);
  GemmPlan plan = plan_gemm(M, N, K, math);
  if (plan.tile && !(va && vb)) plan = GemmPlan{0, K > 0 ? choose_split(M, N, K) : 1};
  const int tile = plan.tile;
  int S = plan.S;
  if (S > 1 && (ws == nullptr || ws_floats < (size_t)S * M * N + (size_t)S * M)) S = 1;
  const int kchunk = S > 1 ? cdiv(cdiv(K, S), BK) * BK : (K > 0 ? K : 1);
  S = K > 0 ? cdiv(K, kchunk) : 1;
  const int bm = tile == 2 ? 256 : BM, bn = tile == 1 ? 256 : BN;
  dim3 grid(cdiv(N, bn), cdiv(M, bm), S);
  float* part = S > 1 ? ws : nullptr;
  float* rowpart = (S > 1 && rowsum) ? ws + (size_t)S * M * N : nullptr;
  const PendEpi pe = take_pending();   // a deferred epilogue rides in this launch
  PAIG_REQUIRE(!pe.S || !part || (pe.part != part && pe.rowpart != part),
               "paig_gemm_ex: the deferred epilogue's partial slabs share this GEMM's workspace");
#define PAIG_G(TA_, TB_)                                                                                       \
  launch_gemm<TA_, TB_>(math, tile, grid, st, M, N, K, kchunk, alpha, A, lda, va, B, ldb, vb, C, ldc, beta, bias, act, auxm, \
                        aux, ldaux, part, rowsum, rowpart, pe)
  if (ta && tb) PAIG_G(true, true);
  else if (ta) PAIG_G(true, false);
  else if (tb) PAIG_G(false, true);
  else PAIG_G(false, false);
#undef PAIG_G
  PAIG_CHECK_LAUNCH();
  if (S > 1) {
    const PendEpi e = make_epi(M, N, S, part, C, ldc, beta, bias, act, auxm, aux, ldaux, rowpart, rowsum);
    if (defer) {
      g_pend = e;   // the next paig_gemm_ex launch carries it
    } else {
      launch_epi(e, st);
      PAIG_CHECK_LAUNCH();
    }
  }
  return 0;
}

}  // extern "C"

PAIG_F16_RANGE_ACCESSOR(paig_f16_range_gemm)
