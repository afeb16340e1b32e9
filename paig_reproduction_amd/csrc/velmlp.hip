// Velocity encoder MLP, fused (reference VelocityEncoder, nn/network/blocks.py:
// 22-29 and forward :43-48: object-split rows [K*B, 2*S] -> Linear(2S,100)
// -> tanh -> Linear(100,100) -> tanh -> Linear(100,2)).
//
// 200 rows x 100 hidden units: six dependent GEMM launches of a few
// microseconds each are pure latency, so the whole forward is ONE launch (row
// blocks; the input packing of blocks.py:43-45 fused in), and the whole
// backward is ONE launch writing per-block partial [W0|b0|W2|b2|W4|b4]
// gradients (the parameters' flat-buffer order) for the step's batched
// deterministic slab reduction.
#include "common.h"
#include "vfn.h"

namespace {

constexpr int HID = 100, OUT = 2, RB = 1, MAXIN = 16;   // RB: backward rows per block (200 blocks at B = 100)
typedef float f32x4v __attribute__((ext_vector_type(4)));

// X[r][2t+j] = pos[b][t][2k+j], r = k*B + b (the chunk/cat of blocks.py:43-45)
__device__ __forceinline__ float packed_in(const float* pos, int B, int Te, int K, int r, int col) {
  const int k = r / B, b = r % B, t = col >> 1, j = col & 1;
  return pos[((long long)b * Te + t) * 2 * K + 2 * k + j];
}

// forward rows per block: 1 (200 blocks for the 200 rows of spring B=100),
// so the per-thread hidden-layer loop is short; W2 is staged per block into
// LDS with an odd row pitch (lanes walk different rows: conflict-free)
constexpr int FRB = 1, W2P = HID + 1;

struct VelFwd {
  const float* pos;
  int B, Te, K, IN;
  const float *W0, *b0, *W2, *b2, *W4, *b4;
  float *X, *h1, *h2, *vel;
};

// one row block of NTHR (>= 128) threads
template <int NTHR>
__device__ __forceinline__ void velmlp_fwd_block(const VelFwd& a, int blk) {
  const float* __restrict__ pos = a.pos;
  const int B = a.B, Te = a.Te, K = a.K, IN = a.IN;
  const float* __restrict__ W0 = a.W0;
  const float* __restrict__ b0 = a.b0;
  const float* __restrict__ W2 = a.W2;
  const float* __restrict__ b2 = a.b2;
  const float* __restrict__ W4 = a.W4;
  const float* __restrict__ b4 = a.b4;
  float* __restrict__ X = a.X;
  float* __restrict__ h1 = a.h1;
  float* __restrict__ h2 = a.h2;
  float* __restrict__ vel = a.vel;
  __shared__ float Xs[FRB][MAXIN];
  __shared__ float H1[HID][FRB], H2[FRB][HID + 1];   // H1 [u][r]: one broadcast read per u
  __shared__ float W2s[HID * W2P];
  const int rows = K * B, r0 = blk * FRB, tid = threadIdx.x;
  const int nr = rows - r0 < FRB ? rows - r0 : FRB;
  const int lane = tid & 63, wv = tid >> 6;
  // every parameter this thread needs is loaded up front, beside W2, so the
  // block pays ONE memory round trip (the layers used to load W0 / b0, b2
  // and W4 / b4 after their barriers: three dependent trips)
  float w[MAXIN], bb0 = 0.f, bb2 = 0.f;
  if (tid < HID) {
    for (int i = 0; i < IN; ++i) w[i] = W0[tid * IN + i];
    bb0 = b0[tid];
    bb2 = b2[tid];
  }
  // output layer: wave wv owns output wv (FRB * OUT == 2 outputs, 2 waves)
  static_assert(FRB * OUT <= 2, "one output per wave");
  const int jo = wv % OUT;
  const float w4a = W4[jo * HID + lane], w4b = lane + 64 < HID ? W4[jo * HID + lane + 64] : 0.f, bb4 = b4[jo];
  if (((uintptr_t)W2 & 15) == 0) {   // all of W2 in flight at once: 20 float4 per thread
#pragma unroll 5
    for (int e = tid; e < HID * HID / 4; e += NTHR) {
      const f32x4v v = reinterpret_cast<const f32x4v*>(W2)[e];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = 4 * e + j;
        W2s[(q / HID) * W2P + q % HID] = v[j];
      }
    }
  } else {
#pragma unroll 8
    for (int q = tid; q < HID * HID; q += NTHR) W2s[(q / HID) * W2P + q % HID] = W2[q];
  }
  for (int e = tid; e < nr * IN; e += blockDim.x) {
    const int r = e / IN, c = e % IN;
    const float v = packed_in(pos, B, Te, K, r0 + r, c);
    Xs[r][c] = v;
    X[(long long)(r0 + r) * IN + c] = v;
  }
  __syncthreads();
  if (tid < HID) {
#pragma unroll
    for (int r = 0; r < FRB; ++r) {
      float a = 0.f;
      if (r < nr) {
        a = bb0;
        for (int i = 0; i < IN; ++i) a = fmaf(Xs[r][i], w[i], a);
        a = tanhf(a);
        h1[(long long)(r0 + r) * HID + tid] = a;
      }
      H1[tid][r] = a;   // ragged last block: zeros
    }
  }
  __syncthreads();
  if (tid < HID) {
    float a[FRB];
#pragma unroll
    for (int r = 0; r < FRB; ++r) a[r] = bb2;
    const float* wr = W2s + tid * W2P;
#pragma unroll 10
    for (int u = 0; u < HID; ++u) {
      const float w = wr[u];
#pragma unroll
      for (int r = 0; r < FRB; ++r) a[r] = fmaf(H1[u][r], w, a[r]);
    }
    for (int r = 0; r < nr; ++r) {
      const float v = tanhf(a[r]);
      H2[r][tid] = v;
      h2[(long long)(r0 + r) * HID + tid] = v;
    }
  }
  __syncthreads();
  // vel[r][j]: one wave per output, lanes split the hidden units (the same
  // two-term order per lane as a stride-64 loop)
  if (wv < nr * OUT) {
    const int r = wv / OUT;
    float a = fmaf(H2[r][lane], w4a, 0.f);
    if (lane + 64 < HID) a = fmaf(H2[r][lane + 64], w4b, a);
    a = wave_sum(a);
    if (lane == 0) vel[(long long)(r0 + r) * OUT + jo] = a + bb4;
  }
}

__global__ void __launch_bounds__(128) velmlp_fwd_k(VelFwd a) { velmlp_fwd_block<128>(a, blockIdx.x); }

// the velocity MLP's row blocks and the VariableFromNetwork forward's blocks
// (independent computations) in ONE launch of 256-thread blocks: on the
// step's single stream every launch saved is time saved
__global__ void __launch_bounds__(256) velmlp_vfn_fwd_k(VelFwd a, int nvel, paig_vfn::VfnFwdTasks T) {
  if ((int)blockIdx.x < nvel) velmlp_fwd_block<256>(a, blockIdx.x);
  else paig_vfn::vfn_fwd_block(T, blockIdx.x - nvel);
}

// slab row (per block): [W0 (HID*IN) | b0 (HID) | W2 (HID*HID) | b2 (HID) | W4 (OUT*HID) | b4 (OUT)]
__global__ void __launch_bounds__(256)
velmlp_bwd_k(const float* __restrict__ dvel, const float* __restrict__ X, const float* __restrict__ h1,
             const float* __restrict__ h2, const float* __restrict__ W0, const float* __restrict__ W2,
             const float* __restrict__ W4, float* __restrict__ dX, float* __restrict__ slab, int rows, int IN) {
  __shared__ float Xs[RB][MAXIN], DV[RB][OUT];
  __shared__ float H1[RB][HID + 1], DZ2[RB][HID + 1], DZ1[RB][HID + 1];
  __shared__ __attribute__((aligned(16))) float W2s[HID * HID];   // read in the dz1 loop
  __shared__ float W0s[HID * MAXIN];                               // read in the dX loop
  const int r0 = blockIdx.x * RB, tid = threadIdx.x;
  const int nr = rows - r0 < RB ? rows - r0 : RB;
  const long long len = (long long)HID * IN + HID + HID * HID + HID + OUT * HID + OUT;
  float* s = slab + blockIdx.x * len;
  float* sW0 = s;
  float* sb0 = sW0 + HID * IN;
  float* sW2 = sb0 + HID;
  float* sb2 = sW2 + HID * HID;
  float* sW4 = sb2 + HID;
  float* sb4 = sW4 + OUT * HID;
  // weights staged with all loads in flight (a dependent global load per loop
  // iteration is what a 100-long dot product would otherwise wait on)
  if (((uintptr_t)W2 & 15) == 0) {
#pragma unroll 10
    for (int e = tid; e < HID * HID / 4; e += 256)
      reinterpret_cast<f32x4v*>(W2s)[e] = reinterpret_cast<const f32x4v*>(W2)[e];
  } else {
#pragma unroll 8
    for (int q = tid; q < HID * HID; q += 256) W2s[q] = W2[q];
  }
#pragma unroll 4
  for (int q = tid; q < HID * IN; q += 256) W0s[q] = W0[q];
  for (int e = tid; e < RB * IN; e += blockDim.x) {
    const int r = e / IN, c = e % IN;
    Xs[r][c] = r < nr ? X[(long long)(r0 + r) * IN + c] : 0.f;
  }
#pragma unroll 4
  for (int e = tid; e < RB * HID; e += blockDim.x) {
    const int r = e / HID, u = e % HID;
    H1[r][u] = r < nr ? h1[(long long)(r0 + r) * HID + u] : 0.f;
  }
  if (tid < RB * OUT) DV[tid / OUT][tid % OUT] = tid / OUT < nr ? dvel[(long long)(r0 + tid / OUT) * OUT + tid % OUT] : 0.f;
  // layer 4's operands loaded before the barrier too: the whole block pays
  // one memory round trip
  float w4[OUT], hvr[RB];
  if (tid < HID) {
#pragma unroll
    for (int j = 0; j < OUT; ++j) w4[j] = W4[j * HID + tid];
#pragma unroll
    for (int r = 0; r < RB; ++r) hvr[r] = r < nr ? h2[(long long)(r0 + r) * HID + tid] : 0.f;
  }
  __syncthreads();
  // ---- layer 4 (linear): dz2 = (dvel W4) * tanh'(h2);  gW4 = dvel^T h2, gb4 = sum dvel
  if (tid < HID) {
    float g4[OUT] = {0.f, 0.f};
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const float hv = hvr[r];
      float d = 0.f;
#pragma unroll
      for (int j = 0; j < OUT; ++j) {
        d = fmaf(DV[r][j], w4[j], d);
        g4[j] = fmaf(DV[r][j], hv, g4[j]);
      }
      DZ2[r][tid] = d * (1.f - hv * hv);
    }
#pragma unroll
    for (int j = 0; j < OUT; ++j) sW4[j * HID + tid] = g4[j];
  }
  if (tid < OUT) {
    float a = 0.f;
    for (int r = 0; r < RB; ++r) a += DV[r][tid];
    sb4[tid] = a;
  }
  __syncthreads();
  // ---- layer 2: gW2[t][u] = sum_r dz2[r][t] h1[r][u], gb2 = sum dz2
  for (int e = tid; e < HID * HID; e += blockDim.x) {
    const int t = e / HID, u = e % HID;
    float a = 0.f;
#pragma unroll
    for (int r = 0; r < RB; ++r) a = fmaf(DZ2[r][t], H1[r][u], a);
    sW2[e] = a;
  }
  if (tid < HID) {
    float a = 0.f;
    for (int r = 0; r < RB; ++r) a += DZ2[r][tid];
    sb2[tid] = a;
    // dz1[r][u = tid] = (sum_t dz2[r][t] W2[t][u]) * tanh'(h1)
    float d[RB];
    for (int r = 0; r < RB; ++r) d[r] = 0.f;
#pragma unroll 4
    for (int t = 0; t < HID; ++t) {
      const float w = W2s[t * HID + tid];
#pragma unroll
      for (int r = 0; r < RB; ++r) d[r] = fmaf(DZ2[r][t], w, d[r]);
    }
    for (int r = 0; r < RB; ++r) DZ1[r][tid] = d[r] * (1.f - H1[r][tid] * H1[r][tid]);
  }
  __syncthreads();
  // ---- layer 0: gW0[u][i] = sum_r dz1[r][u] X[r][i], gb0 = sum dz1, dX = dz1 W0
  for (int e = tid; e < HID * IN; e += blockDim.x) {
    const int u = e / IN, i = e % IN;
    float a = 0.f;
#pragma unroll
    for (int r = 0; r < RB; ++r) a = fmaf(DZ1[r][u], Xs[r][i], a);
    sW0[e] = a;
  }
  if (tid < HID) {
    float a = 0.f;
    for (int r = 0; r < RB; ++r) a += DZ1[r][tid];
    sb0[tid] = a;
  }
  for (int e = tid; e < nr * IN; e += blockDim.x) {
    const int r = e / IN, i = e % IN;
    float a = 0.f;
#pragma unroll 4
    for (int u = 0; u < HID; ++u) a = fmaf(DZ1[r][u], W0s[u * IN + i], a);
    dX[(long long)(r0 + r) * IN + i] = a;
  }
}

}  // namespace

extern "C" {

int paig_velmlp_fwd(const float* pos, int B, int Te, int K, int S, const float* W0, const float* b0, const float* W2,
                    const float* b2, const float* W4, const float* b4, float* X, float* h1, float* h2, float* vel,
                    void* stream) {
  const int IN = 2 * S, rows = K * B;
  if (rows <= 0) return 0;
  PAIG_REQUIRE(IN <= MAXIN && S <= Te, "velmlp: input_steps %d unsupported (max %d)", S, MAXIN / 2);
  const VelFwd a{pos, B, Te, K, IN, W0, b0, W2, b2, W4, b4, X, h1, h2, vel};
  hipLaunchKernelGGL(velmlp_fwd_k, dim3(cdiv(rows, FRB)), dim3(128), 0, (hipStream_t)stream, a);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_velmlp_vfn_fwd(const float* pos, int B, int Te, int K, int S, const float* W0, const float* b0,
                        const float* W2, const float* b2, const float* W4, const float* b4, float* X, float* h1,
                        float* h2, float* vel, int n, const float* const* vW1, const float* const* vb1,
                        const float* const* vW2, const float* const* vb2, float* const* hout, float* const* y,
                        float* const* ypost, const int* P, void* stream) {
  const int IN = 2 * S, rows = K * B;
  PAIG_REQUIRE(rows > 0 && IN <= MAXIN && S <= Te, "velmlp_vfn: rows=%d, input_steps %d (max %d)", rows, S,
               MAXIN / 2);
  PAIG_REQUIRE(n >= 1 && n <= paig_vfn::VMAX, "velmlp_vfn: n=%d (1..%d)", n, paig_vfn::VMAX);
  paig_vfn::VfnFwdTasks T;
  const int nv = paig_vfn::vfn_fwd_tasks(T, n, vW1, vb1, vW2, vb2, hout, y, ypost, P);
  const VelFwd a{pos, B, Te, K, IN, W0, b0, W2, b2, W4, b4, X, h1, h2, vel};
  const int nvel = cdiv(rows, FRB);
  hipLaunchKernelGGL(velmlp_vfn_fwd_k, dim3(nvel + nv), dim3(256), 0, (hipStream_t)stream, a, nvel, T);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_velmlp_bwd_blocks(int rows) { return cdiv(rows, RB); }

int paig_velmlp_slab_len(int S) { return HID * 2 * S + HID + HID * HID + HID + OUT * HID + OUT; }

int paig_velmlp_bwd(const float* dvel, const float* X, const float* h1, const float* h2, const float* W0,
                    const float* W2, const float* W4, float* dX, float* slab, int rows, int S, void* stream) {
  const int IN = 2 * S;
  if (rows <= 0) return 0;
  PAIG_REQUIRE(IN <= MAXIN, "velmlp: input_steps %d unsupported", S);
  hipLaunchKernelGGL(velmlp_bwd_k, dim3(cdiv(rows, RB)), dim3(256), 0, (hipStream_t)stream, dvel, X, h1, h2, W0, W2,
                     W4, dX, slab, rows, IN);
  PAIG_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Encoder position head, fused: l3 (Linear(IN=200, 2)) + split/cat + tanh
// (nn/network/blocks.py:100-102).  Rows n = k*F + f of h2 [K*F][IN]:
//   h3[n][j] = b3[j] + h2[n] . W3[j],   pos[f][2k+j] = tanh(h3[n][j]) * half + half
// and its backward (dpos -> dh3 -> dW3/db3 partials + dh2 * relu'(h2)).
namespace {

constexpr int HEAD_RB = 16;   // rows per backward block

__global__ void __launch_bounds__(256)
head_fwd_k(const float* __restrict__ h2, const float* __restrict__ W3, const float* __restrict__ b3,
           float* __restrict__ h3, float* __restrict__ pos, int F, int K, int IN, float half) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);   // one wave per row
  if (n >= K * F) return;
  const float* x = h2 + (long long)n * IN;
  float a0 = 0.f, a1 = 0.f;
  for (int u = lane; u < IN; u += 64) {
    const float v = x[u];
    a0 = fmaf(v, W3[u], a0);
    a1 = fmaf(v, W3[IN + u], a1);
  }
  a0 = wave_sum(a0) + b3[0];
  a1 = wave_sum(a1) + b3[1];
  if (lane == 0) {
    const int k = n / F, f = n % F;
    h3[(long long)n * 2] = a0;
    h3[(long long)n * 2 + 1] = a1;
    pos[(long long)f * 2 * K + 2 * k] = tanhf(a0) * half + half;
    pos[(long long)f * 2 * K + 2 * k + 1] = tanhf(a1) * half + half;
  }
}

// the velocity encoder's input gradient folded into d enc_pos (what
// paig_vel_unpack_add adds, in the same order): dX [K*B][cols] of the packed
// rows, dpos0 [B][2K] of step S-1 (nullable)
struct VelGrad {
  const float* dX;
  const float* dpos0;
  int B, Te, S, alt;
};
__device__ __forceinline__ float vel_grad(const VelGrad& v, int K, int f, int k, int j) {
  const int b = f / v.Te, t = f % v.Te;
  if (v.dX == nullptr && v.dpos0 == nullptr) return 0.f;
  if (t >= v.S) return 0.f;
  const int cols = (v.alt ? v.S - 1 : v.S) * 2;
  float g = 0.f;
  if (v.dX) {
    const float* xr = v.dX + (long long)(k * v.B + b) * cols;
    if (v.alt) {
      if (t >= 1) g += xr[(t - 1) * 2 + j];
      if (t <= v.S - 2) g -= xr[t * 2 + j];
    } else {
      g += xr[t * 2 + j];
    }
  }
  if (v.dpos0 && t == v.S - 1) g += v.dpos0[(long long)b * 2 * K + 2 * k + j];
  return g;
}

// slab row per block: [W3 (2*IN) | b3 (2)]; blk = the block's row block
// (dstash: the block's dh2 rows also go to this LDS array [RB][IN])
template <int RB = HEAD_RB>
__device__ __forceinline__ void head_bwd_block(const float* __restrict__ h2, const float* __restrict__ h3,
                                               const float* __restrict__ dpos, const float* __restrict__ W3,
                                               float* __restrict__ dh2, float* __restrict__ slab, int F, int K,
                                               int IN, float half, const VelGrad& vg, int blk,
                                               float* dstash = nullptr) {
  __shared__ float D3[RB][2];
  const int n0 = blk * RB, rows = K * F, tid = threadIdx.x;
  const int nr = rows - n0 < RB ? rows - n0 : RB;
  // this thread's first column of h2 for all the block's rows, loaded before
  // the head's reduction so the two latencies overlap (a load per row inside
  // the loop below cost one memory round trip per row)
  float xv[RB];
#pragma unroll
  for (int r = 0; r < RB; ++r) xv[r] = tid < IN && r < nr ? h2[(long long)(n0 + r) * IN + tid] : 0.f;
  if (tid < RB * 2) {
    const int r = tid >> 1, j = tid & 1;
    float d = 0.f;
    if (r < nr) {
      const int n = n0 + r, k = n / F, f = n % F;
      const float t = tanhf(h3[(long long)n * 2 + j]);
      const float dp = dpos[(long long)f * 2 * K + 2 * k + j] + vel_grad(vg, K, f, k, j);
      d = dp * half * (1.f - t * t);
    }
    D3[r][j] = d;
  }
  __syncthreads();
  float* s = slab + (long long)blk * (2 * IN + 2);
  for (int u = tid; u < IN; u += blockDim.x) {
    if (u != tid)
#pragma unroll
      for (int r = 0; r < RB; ++r) xv[r] = r < nr ? h2[(long long)(n0 + r) * IN + u] : 0.f;
    const float w0 = W3[u], w1 = W3[IN + u];
    float g0 = 0.f, g1 = 0.f;
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      if (r < nr) {
        const long long o = (long long)(n0 + r) * IN + u;
        const float x = xv[r];
        g0 = fmaf(D3[r][0], x, g0);
        g1 = fmaf(D3[r][1], x, g1);
        const float g = fmaf(D3[r][0], w0, D3[r][1] * w1);
        dh2[o] = x > 0.f ? g : 0.f;                     // relu' of l2's output (blocks.py:99)
        if (dstash) dstash[r * IN + u] = x > 0.f ? g : 0.f;
      }
    }
    s[u] = g0;
    s[IN + u] = g1;
  }
  if (tid < 2) {
    float a = 0.f;
    for (int r = 0; r < nr; ++r) a += D3[r][tid];
    s[2 * IN + tid] = a;
  }
}

__global__ void __launch_bounds__(256)
head_bwd_k(const float* __restrict__ h2, const float* __restrict__ h3, const float* __restrict__ dpos,
           const float* __restrict__ W3, float* __restrict__ dh2, float* __restrict__ slab, int F, int K, int IN,
           float half, VelGrad vg) {
  head_bwd_block(h2, h3, dpos, W3, dh2, slab, F, K, IN, half, vg, blockIdx.x);
}

// the head backward's row blocks and the VariableFromNetwork backward's phase
// 2 (independent: its phase 1 ran earlier on the stream) in one launch; a
// phase-2 block takes 4 items, one per wave
__global__ void __launch_bounds__(256)
head_bwd_vfn2_k(const float* __restrict__ h2, const float* __restrict__ h3, const float* __restrict__ dpos,
                const float* __restrict__ W3, float* __restrict__ dh2, float* __restrict__ slab, int F, int K, int IN,
                float half, VelGrad vg, int nhead, paig_vfn::VfnBwdTasks T, int nitems) {
  if ((int)blockIdx.x < nhead) {
    head_bwd_block(h2, h3, dpos, W3, dh2, slab, F, K, IN, half, vg, blockIdx.x);
  } else {
    const int item = ((int)blockIdx.x - nhead) * 4 + (threadIdx.x >> 6);
    if (item < nitems) paig_vfn::vfn_bwd2_item(T, item, threadIdx.x & 63);
  }
}

// ---------------------------------------------------------------------------
// The localiser's dense tail in one launch each way (nn/network/blocks.py:
// 98-102: l1 -> ReLU -> l2 -> ReLU -> l3 -> tanh head).  The 200-wide l2 is
// 2000 x 200 x 200: as an MFMA GEMM launch it is all latency (7 K-steps,
// 128 tiles), so it runs in fp32 FMA inside the launches around it:
//   forward: l1's split-K slabs summed (+ b1, ReLU; the order of
//     gemm_splitk_epilogue_k) -> h1; h2 = ReLU(h1 W2^T + b2); the l3 head
//     (head_fwd_k's per-row order) -> h3, enc_pos.  8 rows per block.
//   backward: the head backward's blocks (16 rows, dh2 kept in LDS) also form
//     l2's data gradient dh1 = (dh2 W2) * (h1 > 0).
// Plain fp32 FMA throughout: at least as accurate as the split MFMA form.
// Both launches multiply 8 rows by W2 per block (250 blocks at K*F = 2000):
// 512 threads = (column quad, K-slice of TSL): a thread holds its four W2
// rows' (forward, from W2^T) / columns' (backward) slice in registers
// (float4 loads, coalesced over the quads, all issued at once: one L2 round
// trip), reads each h1 / dh2 value once from LDS for all four columns
// (packed fp32 FMA), and the slices' partials are summed in LDS in slice
// order.  IN <= 200 = TNQ quads x TNS slices of TSL.
constexpr int TAIL_RB = 8, TAIL_NT = 512, TSL = 20, TNS = 10, TNQ = 50, TAIL_MAXIN = 4 * TNQ;

// columns c0 .. c0+3 of M [k][IN] over rows k0 .. k0+kn (one float4 per row)
__device__ __forceinline__ void load_quad_slice(const float* __restrict__ M, int IN, int c0, int k0, int kn,
                                                float4* w) {
#pragma unroll
  for (int k = 0; k < TSL; ++k)
    w[k] = k < kn ? *reinterpret_cast<const float4*>(M + (long long)(k0 + k) * IN + c0) : make_float4(0.f, 0.f, 0.f, 0.f);
}

// W2t = W2^T ([IN][IN]; 32 x 32 tiles through LDS)
__global__ void __launch_bounds__(256) transpose_sq_k(const float* __restrict__ A, float* __restrict__ At, int n) {
  __shared__ float T[32][33];
  const int bx = blockIdx.x * 32, by = blockIdx.y * 32, tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int y = ty; y < 32; y += 8)
    if (by + y < n && bx + tx < n) T[y][tx] = A[(long long)(by + y) * n + bx + tx];
  __syncthreads();
  for (int y = ty; y < 32; y += 8)
    if (bx + y < n && by + tx < n) At[(long long)(bx + y) * n + by + tx] = T[tx][y];
}

// acc[r][0..1] += rows r of X (LDS [TAIL_RB][IN], slice k0..k0+kn) x the
// quad's slice w[k] (columns c0 .. c0+3 at row k0 + k)
__device__ __forceinline__ void quad_slice(const float* X, int IN, int k0, int kn, const float4* w, pf32x2 (*acc)[2]) {
#pragma unroll
  for (int j = 0; j < TSL / 4; ++j) {
    if (4 * j < kn) {
#pragma unroll
      for (int r = 0; r < TAIL_RB; ++r) {
        const float4 x = *reinterpret_cast<const float4*>(&X[r * IN + k0 + 4 * j]);
        const float xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 wq = w[4 * j + q];
          acc[r][0] += xs[q] * pf32x2{wq.x, wq.y};
          acc[r][1] += xs[q] * pf32x2{wq.z, wq.w};
        }
      }
    }
  }
}

// the quad's partials of slice ks -> RQ [slice][row][column]
__device__ __forceinline__ void quad_store(float* RQ, int ks, int c0, pf32x2 (*acc)[2]) {
#pragma unroll
  for (int r = 0; r < TAIL_RB; ++r)
    *reinterpret_cast<float4*>(&RQ[(ks * TAIL_RB + r) * TAIL_MAXIN + c0]) =
        make_float4(acc[r][0].x, acc[r][0].y, acc[r][1].x, acc[r][1].y);
}

__global__ void __launch_bounds__(TAIL_NT)
dense_tail_fwd_k(const float* __restrict__ part, int S, const float* __restrict__ b1, float* __restrict__ h1,
                 const float* __restrict__ W2t, const float* __restrict__ b2, float* __restrict__ h2,
                 const float* __restrict__ W3, const float* __restrict__ b3, float* __restrict__ h3,
                 float* __restrict__ pos, int F, int K, int IN, float half) {
  __shared__ __attribute__((aligned(16))) float X1[TAIL_RB * TAIL_MAXIN];
  __shared__ float X2[TAIL_RB * TAIL_MAXIN];
  __shared__ __attribute__((aligned(16))) float RQ[TNS * TAIL_RB * TAIL_MAXIN];
  const int rows = K * F, n0 = blockIdx.x * TAIL_RB, tid = threadIdx.x;
  const int nr = rows - n0 < TAIL_RB ? rows - n0 : TAIL_RB;
  const long long MN = (long long)rows * IN;
  // this thread's W2 rows c0 .. c0+3 over K-slice ks, from W2^T (W2t [k][c]),
  // loaded first (they fly behind the slab sums)
  const int qd = tid % TNQ, ks = tid / TNQ, c0 = 4 * qd, k0 = ks * TSL;
  const bool act = ks < TNS && c0 < IN && k0 < IN;
  const int kn = act ? (IN - k0 < TSL ? IN - k0 : TSL) : 0;
  float4 w[TSL];
  load_quad_slice(W2t, IN, c0, k0, kn, w);
  // h1 = ReLU(sum_s part[s] + b1): slab order, as the split-K epilogue.  A
  // thread's TAIL_E elements x 8 slabs are loaded at once (one round trip
  // per 8 slabs instead of one per element)
  constexpr int TAIL_E = (TAIL_RB * TAIL_MAXIN + TAIL_NT - 1) / TAIL_NT;
  float acc1[TAIL_E];
#pragma unroll
  for (int q = 0; q < TAIL_E; ++q) acc1[q] = 0.f;
  for (int sq = 0; sq < S; sq += 8) {
    float t[TAIL_E][8];
#pragma unroll
    for (int q = 0; q < TAIL_E; ++q) {
      const int e = tid + q * TAIL_NT, r = e / IN, c = e - r * IN;
      const bool ok = e < TAIL_RB * IN && r < nr;
      const float* p = part + (ok ? (long long)(n0 + r) * IN + c : 0);
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) t[q][jj] = ok && sq + jj < S ? p[(sq + jj) * MN] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < TAIL_E; ++q)
#pragma unroll
      for (int jj = 0; jj < 8; ++jj)
        if (sq + jj < S) acc1[q] += t[q][jj];
  }
#pragma unroll
  for (int q = 0; q < TAIL_E; ++q) {
    const int e = tid + q * TAIL_NT, r = e / IN, c = e - r * IN;
    if (e < TAIL_RB * IN) {
      float v = 0.f;
      if (r < nr) {
        v = epi(acc1[q] + b1[c], ACT_RELU, AUX_NONE, nullptr, 0);
        h1[(long long)(n0 + r) * IN + c] = v;
      }
      X1[e] = v;
    }
  }
  __syncthreads();
  // h2 = ReLU(h1 W2^T + b2)
  if (act) {
    pf32x2 acc[TAIL_RB][2];
#pragma unroll
    for (int r = 0; r < TAIL_RB; ++r) acc[r][0] = acc[r][1] = pf32x2{0.f, 0.f};
    quad_slice(X1, IN, k0, kn, w, acc);
    quad_store(RQ, ks, c0, acc);
  }
  __syncthreads();
  const int nsl = (IN + TSL - 1) / TSL;
  for (int e = tid; e < TAIL_RB * IN; e += TAIL_NT) {
    const int r = e / IN, c = e - r * IN;
    float a = 0.f;
    for (int q = 0; q < nsl; ++q) a += RQ[(q * TAIL_RB + r) * TAIL_MAXIN + c];
    const float v = r < nr ? epi(a + b2[c], ACT_RELU, AUX_NONE, nullptr, 0) : 0.f;
    if (r < nr) h2[(long long)(n0 + r) * IN + c] = v;
    X2[e] = v;
  }
  __syncthreads();
  // l3 + tanh head (head_fwd_k's order): wave w takes row w
  const int lane = tid & 63, wv = tid >> 6;
  for (int r = wv; r < nr; r += TAIL_NT / 64) {
    float a0 = 0.f, a1 = 0.f;
    for (int c = lane; c < IN; c += 64) {
      const float v = X2[r * IN + c];
      a0 = fmaf(v, W3[c], a0);
      a1 = fmaf(v, W3[IN + c], a1);
    }
    a0 = wave_sum(a0) + b3[0];
    a1 = wave_sum(a1) + b3[1];
    if (lane == 0) {
      const int n = n0 + r, k = n / F, f = n % F;
      h3[(long long)n * 2] = a0;
      h3[(long long)n * 2 + 1] = a1;
      pos[(long long)f * 2 * K + 2 * k] = tanhf(a0) * half + half;
      pos[(long long)f * 2 * K + 2 * k + 1] = tanhf(a1) * half + half;
    }
  }
}

// head backward (+ the velocity encoder's input gradient) of TAIL_RB rows and
// their l2 data gradient dh1 = (dh2 W2) * (h1 > 0): (column pair, o-slice)
// threads as in the forward, W2's columns read as float2 rows (coalesced);
// and (nvfn > 0) the VariableFromNetwork backward's phase 2 as extra blocks
// (head_bwd_vfn2_k's items, one per wave)
__global__ void __launch_bounds__(TAIL_NT)
head_l2_bwd_k(const float* __restrict__ h2, const float* __restrict__ h3, const float* __restrict__ dpos,
              const float* __restrict__ W3, float* __restrict__ dh2, float* __restrict__ slab, int F, int K, int IN,
              float half, VelGrad vg, const float* __restrict__ W2, const float* __restrict__ h1,
              float* __restrict__ dh1, int nhead, paig_vfn::VfnBwdTasks T, int nitems) {
  __shared__ __attribute__((aligned(16))) float DH[TAIL_RB * TAIL_MAXIN];
  __shared__ __attribute__((aligned(16))) float RQ[TNS * TAIL_RB * TAIL_MAXIN];
  const int tid = threadIdx.x;
  if ((int)blockIdx.x >= nhead) {
    const int item = ((int)blockIdx.x - nhead) * (TAIL_NT / 64) + (tid >> 6);
    if (item < nitems) paig_vfn::vfn_bwd2_item(T, item, tid & 63);
    return;
  }
  const int n0 = blockIdx.x * TAIL_RB, rows = K * F;
  const int nr = rows - n0 < TAIL_RB ? rows - n0 : TAIL_RB;
  // this thread's W2 columns c0 .. c0+3 over o-slice ks (float4 per o)
  const int qd = tid % TNQ, ks = tid / TNQ, c0 = 4 * qd, k0 = ks * TSL;
  const bool act = ks < TNS && c0 < IN && k0 < IN;
  const int kn = act ? (IN - k0 < TSL ? IN - k0 : TSL) : 0;
  float4 w[TSL];
  load_quad_slice(W2, IN, c0, k0, kn, w);
  for (int e = nr * IN + tid; e < TAIL_RB * IN; e += TAIL_NT) DH[e] = 0.f;
  head_bwd_block<TAIL_RB>(h2, h3, dpos, W3, dh2, slab, F, K, IN, half, vg, blockIdx.x, DH);
  __syncthreads();
  if (act) {
    pf32x2 acc[TAIL_RB][2];
#pragma unroll
    for (int r = 0; r < TAIL_RB; ++r) acc[r][0] = acc[r][1] = pf32x2{0.f, 0.f};
    quad_slice(DH, IN, k0, kn, w, acc);
    quad_store(RQ, ks, c0, acc);
  }
  __syncthreads();
  const int nsl = (IN + TSL - 1) / TSL;
  for (int e = tid; e < nr * IN; e += TAIL_NT) {
    const int r = e / IN, c = e - r * IN;
    float a = 0.f;
    for (int q = 0; q < nsl; ++q) a += RQ[(q * TAIL_RB + r) * TAIL_MAXIN + c];
    const long long o = (long long)(n0 + r) * IN + c;
    dh1[o] = epi(a, ACT_NONE, AUX_RELU, h1, o);
  }
}

}  // namespace

extern "C" {

int paig_dense_tail_fwd(const float* part, int S, const float* b1, float* h1, const float* W2, float* W2t,
                        const float* b2, float* h2, const float* W3, const float* b3, float* h3, float* pos, int F,
                        int K, int IN, float half, void* stream) {
  const int rows = K * F;
  if (rows <= 0) return 0;
  PAIG_REQUIRE(S >= 1 && IN > 0 && IN <= TAIL_MAXIN && IN % 4 == 0,
               "dense_tail_fwd: S=%d, IN=%d (<= %d, a multiple of 4)", S, IN, TAIL_MAXIN);
  PAIG_REQUIRE(W2t && (reinterpret_cast<uintptr_t>(W2t) & 15) == 0,
               "dense_tail_fwd: a 16-byte aligned W2t (IN * IN floats) is required");
  if (W2) {   // W2^T into the W2t scratch first (else W2t already holds it: paig_conv_wprep dg = 2)
    hipLaunchKernelGGL(transpose_sq_k, dim3(cdiv(IN, 32), cdiv(IN, 32)), dim3(256), 0, (hipStream_t)stream, W2, W2t,
                       IN);
    PAIG_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(dense_tail_fwd_k, dim3(cdiv(rows, TAIL_RB)), dim3(TAIL_NT), 0, (hipStream_t)stream, part, S, b1, h1,
                     W2t, b2, h2, W3, b3, h3, pos, F, K, IN, half);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_head_l2_bwd(const float* h2, const float* h3, const float* dpos, const float* W3, float* dh2, float* slab,
                     int F, int K, int IN, float half, const float* dX, const float* dpos0, int B, int Te, int S,
                     int alt, const float* W2, const float* h1, float* dh1, int n, const float* const* d,
                     const float* const* y, const int* sig, const float* const* h, const float* const* vW2,
                     float* const* dW1, float* const* db1, float* const* dW2, float* const* db2, float* const* part,
                     const int* P, void* stream) {
  const int rows = K * F;
  if (rows <= 0) return 0;
  PAIG_REQUIRE(IN > 0 && IN <= TAIL_MAXIN && IN % 4 == 0, "head_l2_bwd: IN=%d (<= %d, a multiple of 4)", IN, TAIL_MAXIN);
  PAIG_REQUIRE(W2 && h1 && dh1 && (reinterpret_cast<uintptr_t>(W2) & 15) == 0,
               "head_l2_bwd: W2 (16-byte aligned: float4 loads), h1 and dh1 are required");
  PAIG_REQUIRE((dX == nullptr && dpos0 == nullptr) || (B > 0 && Te > 0 && F == B * Te && S <= Te),
               "head_l2_bwd: F=%d != B=%d x Te=%d or S=%d > Te", F, B, Te, S);
  PAIG_REQUIRE(n >= 0 && n <= paig_vfn::VMAX, "head_l2_bwd: n=%d (0..%d)", n, paig_vfn::VMAX);
  paig_vfn::VfnBwdTasks T{};
  if (n > 0) paig_vfn::vfn_bwd_tasks(T, n, d, y, sig, h, vW2, dW1, db1, dW2, db2, part, P);
  const int nhead = cdiv(rows, TAIL_RB), nitems = paig_vfn::VH * n;
  const VelGrad vg = (dX || dpos0) ? VelGrad{dX, dpos0, B, Te, S, alt} : VelGrad{nullptr, nullptr, 1, 1, 0, 0};
  hipLaunchKernelGGL(head_l2_bwd_k, dim3(nhead + cdiv(nitems, TAIL_NT / 64)), dim3(TAIL_NT), 0, (hipStream_t)stream, h2,
                     h3, dpos, W3,
                     dh2, slab, F, K, IN, half, vg, W2, h1, dh1, nhead, T, nitems);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_head_fwd(const float* h2, const float* W3, const float* b3, float* h3, float* pos, int F, int K, int IN,
                  float half, void* stream) {
  const int rows = K * F;
  if (rows <= 0) return 0;
  hipLaunchKernelGGL(head_fwd_k, dim3(cdiv(rows, 4)), dim3(256), 0, (hipStream_t)stream, h2, W3, b3, h3, pos, F, K, IN,
                     half);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_head_bwd_blocks(int rows) { return cdiv(rows, HEAD_RB); }

int paig_head_l2_bwd_blocks(int rows) { return cdiv(rows, TAIL_RB); }

int paig_head_bwd(const float* h2, const float* h3, const float* dpos, const float* W3, float* dh2, float* slab, int F,
                  int K, int IN, float half, void* stream) {
  const int rows = K * F;
  if (rows <= 0) return 0;
  hipLaunchKernelGGL(head_bwd_k, dim3(cdiv(rows, HEAD_RB)), dim3(256), 0, (hipStream_t)stream, h2, h3, dpos, W3, dh2,
                     slab, F, K, IN, half, VelGrad{nullptr, nullptr, 1, 1, 0, 0});
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_head_bwd_vel_vfn2(const float* h2, const float* h3, const float* dpos, const float* W3, float* dh2,
                           float* slab, int F, int K, int IN, float half, const float* dX, const float* dpos0, int B,
                           int Te, int S, int alt, int n, const float* const* d, const float* const* y,
                           const int* sig, const float* const* h, const float* const* W2, float* const* dW1,
                           float* const* db1, float* const* dW2, float* const* db2, float* const* part, const int* P,
                           void* stream) {
  const int rows = K * F;
  PAIG_REQUIRE(rows > 0 && B > 0 && Te > 0 && F == B * Te && S <= Te,
               "head_bwd_vel_vfn2: F=%d != B=%d x Te=%d or S=%d > Te", F, B, Te, S);
  PAIG_REQUIRE(n >= 1 && n <= paig_vfn::VMAX, "head_bwd_vel_vfn2: n=%d (1..%d)", n, paig_vfn::VMAX);
  paig_vfn::VfnBwdTasks T;
  paig_vfn::vfn_bwd_tasks(T, n, d, y, sig, h, W2, dW1, db1, dW2, db2, part, P);
  const int nhead = cdiv(rows, HEAD_RB), nitems = paig_vfn::VH * n;
  hipLaunchKernelGGL(head_bwd_vfn2_k, dim3(nhead + cdiv(nitems, 4)), dim3(256), 0, (hipStream_t)stream, h2, h3, dpos,
                     W3, dh2, slab, F, K, IN, half, VelGrad{dX, dpos0, B, Te, S, alt}, nhead, T, nitems);
  PAIG_CHECK_LAUNCH();
  return 0;
}

int paig_head_bwd_vel(const float* h2, const float* h3, const float* dpos, const float* W3, float* dh2, float* slab,
                      int F, int K, int IN, float half, const float* dX, const float* dpos0, int B, int Te, int S,
                      int alt, void* stream) {
  const int rows = K * F;
  if (rows <= 0) return 0;
  PAIG_REQUIRE(B > 0 && Te > 0 && F == B * Te && S <= Te, "head_bwd_vel: F=%d != B=%d x Te=%d or S=%d > Te", F, B,
               Te, S);
  hipLaunchKernelGGL(head_bwd_k, dim3(cdiv(rows, HEAD_RB)), dim3(256), 0, (hipStream_t)stream, h2, h3, dpos, W3, dh2,
                     slab, F, K, IN, half, VelGrad{dX, dpos0, B, Te, S, alt});
  PAIG_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
