// Dense layers on pre-split operands (the encoder's localiser MLP l1 / l2,
// nn/network/blocks.py:71-75,98-100, forward, weight gradient and data
// gradient; the velocity encoder's linear layer).
//
// The split-precision GEMM of gemm.hip converts every fp32 operand tile into
// f16 hi + lo pieces inside the GEMM, once per output tile that reads it: the
// l1 projection converted its 3072 x 200 weight 32 times per launch and its
// data gradient converted both operands ~20 M times, so those launches were
// bound by that VALU work (13 VALU per MFMA) and their barriers, at 0.05-0.1 of
// HBM.  Here every operand is split ONCE per step into a "PS image" and the
// GEMM does nothing but fragment loads and MFMAs:
//
//   PS image of a logical matrix X[R][K] (R rows, reduction dim K):
//     hi plane  short[KB][RP/16][4][16][8]   f16 bits of  rn16(2^e_r X[r][k])
//     lo plane  (the same)                   f16 bits of  rn16(2^e_r X[r][k] - hi)
//     element (r, k) at [k/32][r/16][(k%32)/8][r%16][k%8]: the MFMA fragment of
//     16 rows x 32 k (lane l: row l % 16, k 8 (l / 16) ..) is 1 KB with lane l's
//     16 bytes at byte 16 l: a lane-linear, full-line load
//     exps      int[RP]             e_r: max_k |X[r][k]| 2^e_r in [2^14, 2^15)
//                                   (any finite row, subnormal maxima included)
//   and, on request, the fp32 row sums sum_k X[r][k] (fixed order) into a
//   separate vector (the bias gradient of a weight-gradient GEMM's dY^T).
//   RP = R rounded up to 128, KB = ceil(K / 32); padding rows / k are zeros,
//   and so is one extra k-block KB (the GEMM's branch-free ring reads it past
//   the end of its k-range).
//
// Per-row exponents make every element keep 22 significant bits (or an error
// below 2^-40 of its row's largest) whatever the rows' relative magnitudes,
// and a row's pieces do not depend on the other rows: a forward or data-
// gradient row is computed the same way whatever the batch (the data-parallel
// identity of tests/test_gpu_fullsize.py holds exactly for them).
//
// The MFMA fragment of v_mfma_f32_16x16x32_f16 (lane l: row l % 16, k = 8 (l /
// 16) .. + 7) is 16 contiguous bytes of a PS plane at byte 16 l of a 1 KB
// block (lane-linear: fragment-ordered [row][k] images cost the TA 2x): the GEMM loads fragments straight from
// global memory (L2 / L1 shared by the waves that re-read a panel), no LDS,
// no barriers.  One wave owns one output tile; C = sum over k-blocks of
//   lo(A) hi(B) + hi(A) lo(B) + hi(A) hi(B)   (fp32 accumulation)
// times 2^-(e_m + e_n) in the epilogue (exact).
#include "common.h"

#include <cstdlib>

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int PS_RALIGN = 128;   // >= the GEMM block tile

struct PSView {
  const short* hi;
  const short* lo;
  const int* ex;
  int RP;
};

// one PS image: [hi plane][lo plane][exps RP ints][stats 2 x KC x RP floats:
// per-256-k-chunk partial maxima / sums of row-strided sources (scratch)]
constexpr int PS_KCH = 256;
struct PSLayout {
  long long RP, KB, KC, hi_off, lo_off, ex_off, st_off, bytes;
  __host__ __device__ PSLayout(int R, int K) {
    RP = (R + PS_RALIGN - 1) / PS_RALIGN * PS_RALIGN;
    KB = (K + 31) / 32;
    KC = (K + PS_KCH - 1) / PS_KCH;
    const long long plane = RP * (KB + 1) * 32 * 2;
    hi_off = 0;
    lo_off = plane;
    ex_off = 2 * plane;
    st_off = ex_off + RP * 4;
    bytes = st_off + 2 * KC * RP * 4;
  }
};

// ---------------------------------------------------------------- splitting
// One job: op(X)[r][k] = src[r * sr + k * sk] (sk == 1: rows contiguous in k;
// sr == 1: a row's elements strided by sk), R x K, into the image at dst.
struct SplitJob {
  const float* src;
  long long sr, sk;
  int R, K;
  char* dst;
  float* rs;   // row sums (R floats) or null
};
constexpr int MAXJ = 8;
struct SplitJobs {
  SplitJob j[MAXJ];
  int first[MAXJ + 1];   // each job's first block of the launch
  int n;
};

// e with m 2^e in [2^14, 2^15) for any finite m > 0 (subnormals included: no
// clamp; the scaling below is an exact ldexp), 0 for m == 0
__device__ __forceinline__ int ps_exp(float m) {
  const int b = __builtin_bit_cast(int, m);
  return b > 0 ? 141 - ((b >> 23) & 255) : 0;
}
__device__ __forceinline__ float sc2(float v, int e) { return __builtin_amdgcn_ldexpf(v, e); }

// element (r, k) of a plane (halfs): [k/32][r/16][(k%32)/8][r%16][k%8]
__device__ __forceinline__ long long ps_off(long long RP, int r, int k) {
  return ((((long long)(k >> 5) * (RP >> 4) + (r >> 4)) * 4 + ((k >> 3) & 3)) * 16 + (r & 15)) * 8 + (k & 7);
}

__device__ __forceinline__ void split_store4(short* hi, short* lo, long long o, f32x4 v, int e) {
  const HiLo a = split_pk(sc2(v[0], e), sc2(v[1], e)), b = split_pk(sc2(v[2], e), sc2(v[3], e));
  *reinterpret_cast<uint2*>(hi + o) = make_uint2(a.h, b.h);
  *reinterpret_cast<uint2*>(lo + o) = make_uint2(a.l, b.l);
}

// k-contiguous rows: one wave per row, 4 consecutive k per lane, NV float4
// per lane per pass; pass 1 the row's max / sum (wave reductions), pass 2
// re-reads it (L1 / L2) and stores 8-byte pieces
template <int NV>
__device__ void split_rows_kc(const SplitJob& J, int blk, int nblk) {
  const PSLayout Ly(J.R, J.K);
  short* hi = reinterpret_cast<short*>(J.dst + Ly.hi_off);
  short* lo = reinterpret_cast<short*>(J.dst + Ly.lo_off);
  int* ex = reinterpret_cast<int*>(J.dst + Ly.ex_off);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool vec = (J.K % 4 == 0) && ((uintptr_t)J.src % 16 == 0) && (J.sr % 4 == 0);
  const int KP = (int)(Ly.KB + 1) * 32;   // + the zero k-block
  for (int r = blk * 4 + wv; r < Ly.RP; r += nblk * 4) {
    const float* row = J.src + (long long)(r < J.R ? r : 0) * J.sr;
    auto ld = [&](int k) {
      f32x4 v;
      if (r < J.R && vec && k < J.K) {
        v = *reinterpret_cast<const f32x4*>(row + k);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = (r < J.R && k + i < J.K) ? row[k + i] : 0.f;
      }
      return v;
    };
    float m = 0.f, s = 0.f;
    for (int k0 = 0; k0 < J.K; k0 += NV * 256) {
      f32x4 v[NV];
#pragma unroll
      for (int e = 0; e < NV; ++e) v[e] = ld(k0 + (e * 64 + lane) * 4);
#pragma unroll
      for (int e = 0; e < NV; ++e) {
        m = amax2(amax2(m, v[e][0], v[e][1]), v[e][2], v[e][3]);
        s += (v[e][0] + v[e][1]) + (v[e][2] + v[e][3]);
      }
    }
    m = wave_max_u(m);
    s = wave_sum_dpp(s);
    const int e_r = ps_exp(m);
    for (int k0 = 0; k0 < KP; k0 += NV * 256) {
      f32x4 v[NV];
#pragma unroll
      for (int e = 0; e < NV; ++e) v[e] = ld(k0 + (e * 64 + lane) * 4);
#pragma unroll
      for (int e = 0; e < NV; ++e) {
        const int k = k0 + (e * 64 + lane) * 4;
        if (k < KP) split_store4(hi, lo, ps_off(Ly.RP, r, k), v[e], e_r);
      }
    }
    if (lane == 0) {
      ex[r] = e_r;
      if (J.rs && r < J.R) J.rs[r] = s;
    }
  }
}

// Row-strided sources (sr == 1: consecutive rows adjacent, e.g. W^T or the
// transposed activations / gradients of a weight gradient), two phases.
// Thread t covers rows rq .. rq + 3 (one float4) at k offset kq.
__device__ __forceinline__ f32x4 ld_rc(const SplitJob& J, int r0, int rq, int k) {
  f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool vec = ((uintptr_t)J.src % 16 == 0) && (J.sk % 4 == 0);
  if (k < J.K) {
    const float* p = J.src + (long long)k * J.sk + r0 + rq;
    if (vec && r0 + rq + 3 < J.R) v = *reinterpret_cast<const f32x4*>(p);
    else
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = r0 + rq + i < J.R ? p[i] : 0.f;
  }
  return v;
}

// phase 1: block (64 rows, one 256-k chunk): partial row maxima and sums
// (16 float4 loads in flight per thread) into the image's stats section
__device__ void stats_rc(const SplitJob& J, int blk) {
  const PSLayout Ly(J.R, J.K);
  float* stm = reinterpret_cast<float*>(J.dst + Ly.st_off);
  float* sts = stm + Ly.KC * Ly.RP;
  __shared__ float red[2][16][64];
  const int tid = threadIdx.x, rq = (tid & 15) * 4, kq = tid >> 4;
  const int rb = blk / (int)Ly.KC, kc = blk % (int)Ly.KC;
  const int r0 = rb * 64, k0 = kc * PS_KCH;
  f32x4 v[PS_KCH / 16];
#pragma unroll
  for (int i = 0; i < PS_KCH / 16; ++i) v[i] = ld_rc(J, r0, rq, k0 + kq + 16 * i);
  f32x4 m4 = f32x4{0.f, 0.f, 0.f, 0.f}, s4 = m4;
#pragma unroll
  for (int i = 0; i < PS_KCH / 16; ++i)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      m4[c] = fmaxf(m4[c], fabsf(v[i][c]));
      s4[c] += v[i][c];
    }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    red[0][kq][rq + c] = m4[c];
    red[1][kq][rq + c] = s4[c];
  }
  __syncthreads();
  if (tid < 64) {
    float m = 0.f, s = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      m = fmaxf(m, red[0][q][tid]);
      s += red[1][q][tid];
    }
    stm[(long long)kc * Ly.RP + r0 + tid] = m;
    sts[(long long)kc * Ly.RP + r0 + tid] = s;
  }
}

// phase 2: block (64 rows, one 32-k block): the rows' exponents from the
// partial maxima, split, transposed through LDS, 16-byte stores (64 rows x
// 64 B contiguous per piece)
__device__ void split_rc(const SplitJob& J, int blk) {
  const PSLayout Ly(J.R, J.K);
  short* hi = reinterpret_cast<short*>(J.dst + Ly.hi_off);
  short* lo = reinterpret_cast<short*>(J.dst + Ly.lo_off);
  int* ex = reinterpret_cast<int*>(J.dst + Ly.ex_off);
  const float* stm = reinterpret_cast<const float*>(J.dst + Ly.st_off);
  const float* sts = stm + Ly.KC * Ly.RP;
  __shared__ int se[64];
  __shared__ __attribute__((aligned(16))) short th[64][40], tl[64][40];   // [row][k] (80-B rows)
  const int tid = threadIdx.x, rq = (tid & 15) * 4, kq = tid >> 4;
  const int rb = blk / (int)(Ly.KB + 1), kb = blk % (int)(Ly.KB + 1);   // kb == KB: the zero block
  const int r0 = rb * 64;
  const f32x4 v0 = ld_rc(J, r0, rq, kb * 32 + kq), v1 = ld_rc(J, r0, rq, kb * 32 + kq + 16);
  if (tid < 64) {
    float m = 0.f;
    for (int c = 0; c < Ly.KC; ++c) m = fmaxf(m, stm[(long long)c * Ly.RP + r0 + tid]);
    const int e_r = ps_exp(m);
    se[tid] = e_r;
    if (kb == 0) {
      ex[r0 + tid] = e_r;
      if (J.rs && r0 + tid < J.R) {
        float s = 0.f;
        for (int c = 0; c < Ly.KC; ++c) s += sts[(long long)c * Ly.RP + r0 + tid];
        J.rs[r0 + tid] = s;
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const f32x4 v = h ? v1 : v0;
    const int kk = kq + 16 * h;
#pragma unroll
    for (int i = 0; i < 4; i += 2) {
      const HiLo q = split_pk(sc2(v[i], se[rq + i]), sc2(v[i + 1], se[rq + i + 1]));
      th[rq + i][kk] = (short)(q.h & 0xffff);
      th[rq + i + 1][kk] = (short)(q.h >> 16);
      tl[rq + i][kk] = (short)(q.l & 0xffff);
      tl[rq + i + 1][kk] = (short)(q.l >> 16);
    }
  }
  __syncthreads();
  // thread t: row group t / 64, k-chunk (t / 16) % 4, row t % 16: 4 KB contiguous
  const int r = (tid >> 6) * 16 + (tid & 15), c = ((tid >> 4) & 3) * 8;
  const long long o = ps_off(Ly.RP, r0 + r, kb * 32 + c);
  *reinterpret_cast<s16x8*>(hi + o) = *reinterpret_cast<const s16x8*>(&th[r][c]);
  *reinterpret_cast<s16x8*>(lo + o) = *reinterpret_cast<const s16x8*>(&tl[r][c]);
}

__device__ __forceinline__ int job_of(const SplitJobs& js, int& blk, int& nblk) {
  int j = 0;
  while (j + 1 < js.n && (int)blockIdx.x >= js.first[j + 1]) ++j;
  blk = blockIdx.x - js.first[j];
  nblk = js.first[j + 1] - js.first[j];
  return j;
}

// phase 1 launch: k-contiguous jobs split completely, row-strided jobs
// gather their partial statistics
template <int NV>
__global__ void __launch_bounds__(256) ps_split1_k(SplitJobs js) {
  int blk, nblk;
  const SplitJob& J = js.j[job_of(js, blk, nblk)];
  if (J.sk == 1) split_rows_kc<NV>(J, blk, nblk);
  else stats_rc(J, blk);
}
// phase 2 launch: the row-strided jobs' split
__global__ void __launch_bounds__(256) ps_split2_k(SplitJobs js) {
  int blk, nblk;
  const SplitJob& J = js.j[job_of(js, blk, nblk)];
  split_rc(J, blk);
}

// ---------------------------------------------------------------- the GEMM
__device__ __forceinline__ f32x4 mma(s16x8 a, s16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                0);
}

// Block tile BM x BN (4 waves as 2 x 2, each (BM/2) x (BN/2) = TM x TN MFMA
// tiles), one stage = 2 k-blocks (64 k).  A stage of an operand is BM / 16
// consecutive 1 KB fragment blocks per plane per k-block in the PS image, so
// it is copied to LDS as is (lane-linear 16-byte loads and ds_write_b128,
// every byte fetched once per block instead of once per wave) and each
// fragment is one conflict-free lane-linear ds_read_b128.  The next stage's
// loads are in flight (registers) during the current stage's MFMAs; one LDS
// buffer, two barriers per stage.  Past its k-range a block reads the
// image's zero k-block (branch-free loads).
template <int BM, int BN>
struct PsCfg {
  static constexpr int TM = BM / 32, TN = BN / 32;
  static constexpr int AST = BM * 32 * 2;   // halfs of one plane of one k-block of A
  static constexpr int BST = BN * 32 * 2;   // (sizeof short = 2: BM * 32 halfs per plane)
  // per stage: 2 k-blocks x 2 planes x (BM + BN) x 32 halfs
  static constexpr int STAGE = 2 * 2 * (BM + BN) * 32;   // halfs
  static constexpr int NLD = STAGE * 2 / 16 / 256;          // 16-byte loads per thread
  static constexpr int EPI = 4 * (BM / 2) * (BN / 2 + 4) * 2;   // halfs (float image per wave)
  static constexpr int LDS = (STAGE > EPI ? STAGE : EPI) * 2;   // bytes
};

template <int BM, int BN>
__global__ void __launch_bounds__(256) psgemm_k(PSView A, PSView B, int M, int N, int KB, int kbc, int tilesN,
                                                int ntiles, float alpha, float* __restrict__ C, long long ldc,
                                                float beta, const float* __restrict__ bias, int act, int auxm,
                                                const float* __restrict__ aux, long long ldaux,
                                                float* __restrict__ part) {
  using Cf = PsCfg<BM, BN>;
  constexpr int TM = Cf::TM, TN = Cf::TN, NLD = Cf::NLD;
  extern __shared__ __attribute__((aligned(16))) short sm[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  int b = blockIdx.x;
  const int nb = gridDim.x;
  if (nb % 8 == 0) b = (b % 8) * (nb / 8) + b / 8;
  const int s = b / ntiles, rem = b % ntiles;
  const int m0 = (rem / tilesN) * BM, n0 = (rem % tilesN) * BN;
  const int kb0 = s * kbc, kb1 = min(KB, kb0 + kbc);

  // this thread's 16-byte loads of a stage: linear index u = tid + 256 l over
  // [k-block 0 / 1][A hi, A lo, B hi, B lo][rows x 32 halfs]
  auto src = [&](int kbs, int u) -> const s16x8* {
    constexpr int PA = BM * 32 / 8, PB = BN * 32 / 8;   // 16-byte units per plane
    constexpr int PER = 2 * PA + 2 * PB;
    const int h = u / PER, v = u % PER;
    const int kb = kbs + h < kb1 ? kbs + h : KB;
    if (v < 2 * PA) {
      const short* pl = v < PA ? A.hi : A.lo;
      return reinterpret_cast<const s16x8*>(pl + ((long long)kb * (A.RP >> 4) + (m0 >> 4)) * 512) + v % PA;
    }
    const int w = v - 2 * PA;
    const short* pl = w < PB ? B.hi : B.lo;
    return reinterpret_cast<const s16x8*>(pl + ((long long)kb * (B.RP >> 4) + (n0 >> 4)) * 512) + w % PB;
  };
  s16x8 rg[NLD];
  auto issue = [&](int kbs) {
#pragma unroll
    for (int l = 0; l < NLD; ++l) rg[l] = *src(kbs, tid + 256 * l);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue(kb0);
  for (int kbs = kb0; kbs < kb1; kbs += 2) {
    __syncthreads();   // the previous stage's fragment reads are done
#pragma unroll
    for (int l = 0; l < NLD; ++l) reinterpret_cast<s16x8*>(sm)[tid + 256 * l] = rg[l];
    __syncthreads();
    issue(kbs + 2);   // (past the range: zero-block loads, never used)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const short* st = sm + h * 2 * (BM + BN) * 32;
      const short* ahp = st + (wm * (BM / 2)) * 32 + lane * 8;
      const short* alp = ahp + BM * 32;
      const short* bhp = st + 2 * BM * 32 + (wn * (BN / 2)) * 32 + lane * 8;
      const short* blp = bhp + BN * 32;
      s16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        ah[i] = *reinterpret_cast<const s16x8*>(ahp + i * 512);
        al[i] = *reinterpret_cast<const s16x8*>(alp + i * 512);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        bh[j] = *reinterpret_cast<const s16x8*>(bhp + j * 512);
        bl[j] = *reinterpret_cast<const s16x8*>(blp + j * 512);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = mma(al[i], bh[j], acc[i][j]);
          acc[i][j] = mma(ah[i], bl[j], acc[i][j]);
          acc[i][j] = mma(ah[i], bh[j], acc[i][j]);
        }
    }
  }
  __syncthreads();   // the staging LDS becomes the epilogue image

  // epilogue: 2^-(e_m + e_n), then partials or bias / act / aux'.  The wave's
  // tile goes through LDS so each store instruction writes whole 128-B row
  // segments (float4 per lane) instead of 4 rows x 64 B of scattered dwords
  // (the accumulator layout): the stores of the 24.6 MB l1 data gradient and
  // of the split-K partials dominated the scattered form.
  constexpr int TR = BM / 2, TC = BN / 2, LP = TC + 4;
  float* img = reinterpret_cast<float*>(sm) + wv * TR * LP;
  const int wm0 = m0 + wm * TR, wn0 = n0 + wn * TC;
  int en[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) en[j] = B.ex[wn0 + j * 16 + (lane & 15)];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = i * 16 + (lane >> 4) * 4 + r;
      const int em = A.ex[wm0 + rr];
#pragma unroll
      for (int j = 0; j < TN; ++j)
        img[rr * LP + j * 16 + (lane & 15)] = alpha * __builtin_amdgcn_ldexpf(acc[i][j][r], -(em + en[j]));
    }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  constexpr int C4 = TC / 4;   // float4 per tile row
  const bool vec = (N % 4 == 0) && (part || ((ldc % 4 == 0) && ((uintptr_t)C % 16 == 0) &&
                                            (!bias || (uintptr_t)bias % 16 == 0) &&
                                            (auxm == 0 || ((ldaux % 4 == 0) && (uintptr_t)aux % 16 == 0)) &&
                                            beta == 0.f));
#pragma unroll
  for (int q = 0; q < TR * C4 / 64; ++q) {
    const int idx = q * 64 + lane, rr = idx / C4, c = (idx % C4) * 4;
    const int m = wm0 + rr, n = wn0 + c;
    if (m >= M || n >= N) continue;
    f32x4 v = *reinterpret_cast<const f32x4*>(img + rr * LP + c);
    if (vec) {
      if (part) {
        *reinterpret_cast<f32x4*>(part + ((long long)s * M + m) * N + n) = v;
      } else {
        if (bias) v += *reinterpret_cast<const f32x4*>(bias + n);
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = epi(v[e], act, auxm, aux, (long long)m * ldaux + n + e);
        *reinterpret_cast<f32x4*>(C + (long long)m * ldc + n) = o;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (n + e >= N) break;
        float x = v[e];
        if (part) {
          part[((long long)s * M + m) * N + n + e] = x;
        } else {
          if (beta != 0.f) x += beta * C[(long long)m * ldc + n + e];
          if (bias) x += bias[n + e];
          C[(long long)m * ldc + n + e] = epi(x, act, auxm, aux, (long long)m * ldaux + n + e);
        }
      }
    }
  }
}

// k-blocks per split: the split depends on K alone (a forward / data-gradient
// row's sum order does not change with M: the data-parallel identity), 12
// k-blocks (384 k) per wave, no split up to 16
int ps_kchunk(int KB, int /*tiles*/) { return KB <= 16 ? KB : 12; }

}  // namespace

extern "C" {

long long paig_ps_bytes(int R, int K) {
  if (R <= 0 || K <= 0) return 0;
  return PSLayout(R, K).bytes;
}

int paig_ps_split(int n, const float* const* src, const long long* sr, const long long* sk, const int* R,
                  const int* K, void* const* dst, float* const* rowsum, void* stream) {
  if (n <= 0) return 0;
  PAIG_REQUIRE(n <= MAXJ, "paig_ps_split: at most %d jobs per launch, got %d", MAXJ, n);
  SplitJobs j1{}, j2{};
  int t1 = 0, t2 = 0, maxk = 0;
  for (int i = 0; i < n; ++i) {
    PAIG_REQUIRE(R[i] > 0 && K[i] > 0, "paig_ps_split: job %d has R=%d K=%d", i, R[i], K[i]);
    PAIG_REQUIRE(sk[i] == 1 || sr[i] == 1, "paig_ps_split: job %d needs sk == 1 or sr == 1", i);
    PAIG_REQUIRE(((uintptr_t)dst[i]) % 256 == 0, "paig_ps_split: job %d image not 256-byte aligned", i);
    const PSLayout Ly(R[i], K[i]);
    const SplitJob J{src[i], sr[i], sk[i], R[i], K[i], (char*)dst[i], rowsum ? rowsum[i] : nullptr};
    int nb;
    if (sk[i] == 1) {
      maxk = K[i] > maxk ? K[i] : maxk;
      nb = cdiv(Ly.RP, 4);
      if (nb > 2048) nb = 2048;
    } else {
      nb = (int)(Ly.RP / 64 * Ly.KC);
      j2.j[j2.n] = J;
      j2.first[j2.n++] = t2;
      t2 += (int)(Ly.RP / 64 * (Ly.KB + 1));
    }
    j1.j[j1.n] = J;
    j1.first[j1.n++] = t1;
    t1 += nb;
  }
  j1.first[j1.n] = t1;
  j2.first[j2.n] = t2;
  hipStream_t st = (hipStream_t)stream;
  if (maxk <= 256) hipLaunchKernelGGL((ps_split1_k<1>), dim3(t1), dim3(256), 0, st, j1);
  else hipLaunchKernelGGL((ps_split1_k<4>), dim3(t1), dim3(256), 0, st, j1);
  PAIG_CHECK_LAUNCH();
  if (t2 > 0) {
    hipLaunchKernelGGL(ps_split2_k, dim3(t2), dim3(256), 0, st, j2);
    PAIG_CHECK_LAUNCH();
  }
  return 0;
}

// block tile: 128 x 128 where that still gives >= 192 blocks, else 64 x 64;
// PAIG_PS_TILE=1 / 0 in the environment forces one (A/B runs)
static int ps_tile_env() {
  static int v = -2;
  if (v == -2) {
    const char* e = getenv("PAIG_PS_TILE");
    v = e ? atoi(e) : -1;
  }
  return v;
}
struct PSPlan {
  int big, bm, bn, tilesN, tiles, kbc, S;
};
static PSPlan ps_plan(int M, int N, int K) {
  const int KB = (K + 31) / 32;
  const int kbc = ps_kchunk(KB, 0), S = (KB + kbc - 1) / kbc;
  PSPlan p;
  const int e = ps_tile_env();
  p.big = e >= 0 ? e : (cdiv(M, 128) * cdiv(N, 128) * S >= 192);
  p.bm = p.bn = p.big ? 128 : 64;
  p.tilesN = cdiv(N, p.bn);
  p.tiles = cdiv(M, p.bm) * p.tilesN;
  p.kbc = kbc;
  p.S = S;
  return p;
}

size_t paig_psgemm_workspace(int M, int N, int K) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  const PSPlan p = ps_plan(M, N, K);
  return p.S > 1 ? (size_t)p.S * M * N : 0;
}

int paig_psgemm(int M, int N, int K, const void* Aimg, const void* Bimg, float alpha, float* C, long long ldc,
                float beta, const float* bias, int act, int auxm, const float* aux, long long ldaux, float* ws,
                size_t ws_floats, void* stream) {
  if (M <= 0 || N <= 0) return 0;
  PAIG_REQUIRE(K > 0 && Aimg && Bimg, "paig_psgemm: K=%d and both images required", K);
  hipStream_t st = (hipStream_t)stream;
  const PSLayout La(M, K), Lb(N, K);
  const char* a = (const char*)Aimg;
  const char* b = (const char*)Bimg;
  const PSView A{(const short*)(a + La.hi_off), (const short*)(a + La.lo_off), (const int*)(a + La.ex_off),
                 (int)La.RP};
  const PSView B{(const short*)(b + Lb.hi_off), (const short*)(b + Lb.lo_off), (const int*)(b + Lb.ex_off),
                 (int)Lb.RP};
  const int KB = (int)La.KB;
  const PSPlan p = ps_plan(M, N, K);
  float* part = nullptr;
  if (p.S > 1) {
    PAIG_REQUIRE(ws && ws_floats >= (size_t)p.S * M * N, "paig_psgemm: workspace of %zu floats needed",
                 (size_t)p.S * M * N);
    part = ws;
  }
  const dim3 grid(p.tiles * p.S);
  float* Cd = p.S > 1 ? nullptr : C;
  if (p.big) {
    auto k = psgemm_k<128, 128>;
    constexpr int lds = PsCfg<128, 128>::LDS;
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
      attr = true;
    }
    hipLaunchKernelGGL(k, grid, dim3(256), lds, st, A, B, M, N, KB, p.kbc, p.tilesN, p.tiles, alpha, Cd, ldc, beta,
                       bias, act, auxm, aux, ldaux, part);
  } else {
    auto k = psgemm_k<64, 64>;
    constexpr int lds = PsCfg<64, 64>::LDS;
    hipLaunchKernelGGL(k, grid, dim3(256), lds, st, A, B, M, N, KB, p.kbc, p.tilesN, p.tiles, alpha, Cd, ldc, beta,
                       bias, act, auxm, aux, ldaux, part);
  }
  PAIG_CHECK_LAUNCH();
  if (p.S > 1) {
    paig_gemm_splitk_finish(M, N, p.S, part, C, ldc, beta, bias, act, auxm, aux, ldaux, nullptr, nullptr, st);
    PAIG_CHECK_LAUNCH();
  }
  return 0;
}

}  // extern "C"
