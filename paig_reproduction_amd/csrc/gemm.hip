// fp32 GEMM on CDNA4 matrix cores (v_mfma_f32_16x16x4_f32: exact f32 FMA
// chain, same rate as the f32 VALU but one instruction per 16 FMAs/lane).
//
// Used for every dense layer of the path: the encoder's projection to latent
// coordinates (nn/network/blocks.py:71-75,98-100; K = 3072 -> 200, the one
// MFMA-shaped op the north star names), its MLP tail, the velocity MLP
// (blocks.py:23-29) and VariableFromNetwork (blocks.py:311-322), forward and
// backward (dX = dY W, dW = dY^T X).
//
//   C[M,N] = alpha * op(A)[M,K] op(B)[K,N]  (+ beta*C) (+ bias[n]) -> act -> *aux'
//   op(A)[m][k] = TA ? A[k*lda+m] : A[m*lda+k]
//   op(B)[k][n] = TB ? B[n*ldb+k] : B[k*ldb+n]
//
// Tile 64x64x16, 256 threads = 4 waves in 2x2, each wave 32x32 = 2x2 MFMA
// tiles. LDS holds A as [k][m] and B as [k][n] with a 16-float pad so the
// fragment reads (lanes 0-15 one k-row, lanes 16-31 the next) are
// bank-conflict free. Optional split-K writes fp32 partial slabs reduced by
// gemm_splitk_epilogue_k (deterministic).
#include "common.h"

namespace {

constexpr int BM = 64, BN = 64, BK = 16, LDP = 64 + 16;

enum { ACT_NONE = 0, ACT_RELU = 1, ACT_TANH = 2, ACT_SIGMOID = 3 };
enum { AUX_NONE = 0, AUX_RELU = 1, AUX_TANH = 2 };

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float epi(float v, int act, int auxm, const float* aux, long long aoff) {
  if (act == ACT_RELU) v = v < 0.f ? 0.f : v;
  else if (act == ACT_TANH) v = tanhf(v);
  else if (act == ACT_SIGMOID) v = 1.f / (1.f + expf(-v));
  if (auxm == AUX_RELU) v = aux[aoff] > 0.f ? v : 0.f;
  else if (auxm == AUX_TANH) { float t = aux[aoff]; v = v * (1.f - t * t); }
  return v;
}

template <bool TA, bool TB>
__global__ void __launch_bounds__(256)
gemm_k(int M, int N, int K, int kchunk, float alpha, const float* __restrict__ A, long long lda,
       const float* __restrict__ B, long long ldb, float* __restrict__ C, long long ldc, float beta,
       const float* __restrict__ bias, int act, int auxm, const float* __restrict__ aux, long long ldaux,
       float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float As[BK][LDP];
  __shared__ __attribute__((aligned(16))) float Bs[BK][LDP];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int kbeg = blockIdx.z * kchunk;
  int kend = kbeg + kchunk;
  if (kend > K) kend = K;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    // ---- stage A (BM x BK) into As[k][m]
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int idx = tid * 4 + e;  // 0..1023
      int mm, kk;
      if (TA) { kk = idx >> 6; mm = idx & 63; }   // m contiguous in memory
      else { mm = idx >> 4; kk = idx & 15; }      // k contiguous in memory
      const int gm = m0 + mm, gk = k0 + kk;
      float v = 0.f;
      if (gm < M && gk < kend) v = TA ? A[(long long)gk * lda + gm] : A[(long long)gm * lda + gk];
      As[kk][mm] = v;
    }
    // ---- stage B (BK x BN) into Bs[k][n]
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int idx = tid * 4 + e;
      int nn, kk;
      if (TB) { nn = idx >> 4; kk = idx & 15; }   // k contiguous
      else { kk = idx >> 6; nn = idx & 63; }      // n contiguous
      const int gn = n0 + nn, gk = k0 + kk;
      float v = 0.f;
      if (gn < N && gk < kend) v = TB ? B[(long long)gn * ldb + gk] : B[(long long)gk * ldb + gn];
      Bs[kk][nn] = v;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < BK; ks += 4) {
      const int kr = ks + (lane >> 4);
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[kr][wm * 32 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[kr][wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
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
            part[((long long)blockIdx.z * M + m) * N + n] = v;
          } else {
            if (beta != 0.f) v += beta * C[(long long)m * ldc + n];
            if (bias) v += bias[n];
            C[(long long)m * ldc + n] = epi(v, act, auxm, aux, (long long)m * ldaux + n);
          }
        }
      }
}

__global__ void gemm_splitk_epilogue_k(int M, int N, int S, const float* __restrict__ part, float* __restrict__ C,
                                       long long ldc, float beta, const float* __restrict__ bias, int act, int auxm,
                                       const float* __restrict__ aux, long long ldaux) {
  const long long n_el = (long long)M * N;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n_el; i += (long long)gridDim.x * blockDim.x) {
    const int m = (int)(i / N), n = (int)(i % N);
    float v = 0.f;
    for (int s = 0; s < S; ++s) v += part[(long long)s * n_el + i];
    if (beta != 0.f) v += beta * C[(long long)m * ldc + n];
    if (bias) v += bias[n];
    C[(long long)m * ldc + n] = epi(v, act, auxm, aux, (long long)m * ldaux + n);
  }
}

static int choose_split(int M, int N, int K) {
  const int tiles = cdiv(M, BM) * cdiv(N, BN);
  int s = 1;
  while (tiles * s < 512 && K / (s * 2) >= 256) s *= 2;
  return s;
}

}  // namespace

extern "C" {

size_t paig_gemm_workspace(int M, int N, int K) {
  int s = choose_split(M, N, K);
  return s > 1 ? (size_t)s * M * N : 0;
}

int paig_gemm(int ta, int tb, int M, int N, int K, float alpha, const float* A, long long lda, const float* B,
              long long ldb, float beta, float* C, long long ldc, const float* bias, int act, int auxm,
              const float* aux, long long ldaux, float* ws, size_t ws_floats, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (M <= 0 || N <= 0) return 0;
  int S = K > 0 ? choose_split(M, N, K) : 1;
  if (S > 1 && (ws == nullptr || ws_floats < (size_t)S * M * N)) S = 1;
  const int kchunk = S > 1 ? cdiv(cdiv(K, S), BK) * BK : (K > 0 ? K : 1);
  S = K > 0 ? cdiv(K, kchunk) : 1;
  dim3 grid(cdiv(N, BN), cdiv(M, BM), S);
  float* part = S > 1 ? ws : nullptr;
#define PAIG_G(TA_, TB_)                                                                                       \
  hipLaunchKernelGGL((gemm_k<TA_, TB_>), grid, dim3(256), 0, st, M, N, K, kchunk, alpha, A, lda, B, ldb, C, ldc, \
                     beta, bias, act, auxm, aux, ldaux, part)
  if (ta && tb) PAIG_G(true, true);
  else if (ta) PAIG_G(true, false);
  else if (tb) PAIG_G(false, true);
  else PAIG_G(false, false);
#undef PAIG_G
  PAIG_CHECK_LAUNCH();
  if (S > 1) {
    long long n_el = (long long)M * N;
    int g = cdiv(n_el, 256);
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(gemm_splitk_epilogue_k, dim3(g), dim3(256), 0, st, M, N, S, part, C, ldc, beta, bias, act, auxm,
                       aux, ldaux);
    PAIG_CHECK_LAUNCH();
  }
  return 0;
}

}  // extern "C"
