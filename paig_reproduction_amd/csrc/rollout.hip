// Differentiable physics rollout: all R steps x 5 semi-implicit Euler
// substeps in one launch (one thread per sequence), and its adjoint.
//
// Reference cells (nn/network/cells.py):
//   spring_ode_cell.forward   :31-51  (torch.split(x, 1): object "0/1" are the
//                                      columns x0, y0 -- quirk Q3; columns 2,3
//                                      never move)
//   bouncing_ode_cell.forward :60-83  (same split-size-1 quirk, hard walls 0/32)
//   gravity_ode_cell.forward  :96-106 (3 bodies, A = exp(g) exp(2m); computed
//                                      per call here, quirk Q4)
// The rollout loop itself is PhysicsNet.conv_feedforward :231-239.
//
// The reference issues ~100 tiny elementwise ops per step; here each thread
// keeps its sequence's state in registers.  Forward writes pos_vel_seq
// [B][1+R][2D] (which also serves as the decoder's position input).
// Backward recomputes each step's substeps from the stored step-start state
// (no substep storage) and runs the reverse-mode chain; physics-parameter
// gradients are reduced in fp64 per block into a partial slab.
#include "common.h"

namespace {

enum { CELL_SPRING = 0, CELL_BOUNCE = 1, CELL_GRAVITY = 2 };

struct Phys {
  float h;     // dt / 5 (fp32, as torch computes self.dt / 5)
  float ek;    // (float) exp(k)              spring
  float tee;   // (float) (2 * exp(equil))    spring
  float negA;  // (float) -(exp(g) * exp(2m)) gravity
};

// ---------------------------------------------------------------- spring ----
// sqrt(|d*d|) of the reference: in binary IEEE arithmetic with round to
// nearest, sqrt(fl(d*d)) == |d| exactly unless d*d underflows (then 0) or
// overflows (impossible for pixel coordinates) -- one op instead of the IEEE
// sqrt sequence on the rollout's serial chain
__device__ __forceinline__ float abs_via_sq(float d) { return d * d == 0.f ? 0.f : fabsf(d); }

__device__ __forceinline__ void spring_sub(const Phys& P, float* p, float* v) {
  const float d = p[0] - p[1];
  const float n = abs_via_sq(d);
  const float dir = d / (n + 1e-4f);
  const float F = P.ek * (n - P.tee) * dir;
  v[0] = v[0] - P.h * F;
  v[1] = v[1] + P.h * F;
  p[0] = p[0] + P.h * v[0];
  p[1] = p[1] + P.h * v[1];
}

// adjoint of one spring substep, given the substep's INPUT state (p, v).
// gp/gv: adjoints of outputs -> overwritten with adjoints of inputs.
// The adjoint is a long serial chain (46 steps x 5 substeps per thread): its
// divisions use one v_rcp_f32 (1 ulp) instead of the IEEE division sequence,
// and the parameter adjoints accumulate in fp32 within a step (flushed to
// fp64 per step by the caller) -- gradient-side only; the forward keeps the
// reference's exact operations.
__device__ __forceinline__ void spring_sub_bwd(const Phys& P, const float* p, const float* v, float* gp, float* gv,
                                               float& gek, float& gtee) {
  const float d = p[0] - p[1];
  const float dd = d * d;
  const float n = abs_via_sq(d);
  const float den = n + 1e-4f;
  const float rden = __builtin_amdgcn_rcpf(den);
  const float dir = d * rden;
  const float nm = n - P.tee;
  // p' = p + h v'
  gv[0] += P.h * gp[0];
  gv[1] += P.h * gp[1];
  // v0' = v0 - h F ; v1' = v1 + h F
  const float gF = P.h * gv[1] - P.h * gv[0];
  // F = ek * (n - tee) * dir
  gek += gF * nm * dir;
  const float gnm = gF * P.ek * dir;
  gtee -= gnm;
  const float gdir = gF * P.ek * nm;
  // dir = d / (n + 1e-4)
  float gd = gdir * rden;
  float gn = gnm - gdir * d * (rden * rden);
  // n = sqrt(|d*d|)  (aten: sqrt' = g/(2 sqrt), abs' = sgn, pow' = 2d)
  const float gsq = gn * __builtin_amdgcn_rcpf(2.f * n);
  const float sg = dd > 0.f ? 1.f : (dd < 0.f ? -1.f : 0.f);
  gd += gsq * sg * 2.f * d;
  gp[0] += gd;
  gp[1] -= gd;
}

// -------------------------------------------------------------- bouncing ----
__device__ __forceinline__ void bounce_sub(const Phys& P, float* p, float* v, unsigned* fl) {
  p[0] = p[0] + P.h * v[0];
  p[1] = p[1] + P.h * v[1];
  unsigned f = 0;
  for (int j = 0; j < 2; ++j) {
    const bool a = p[j] + 2.f > 32.f;
    if (a) v[j] = -v[j];
    const bool b = 0.f > p[j] - 2.f;
    if (b) v[j] = -v[j];
    if (a) p[j] = 32.f - (p[j] + 2.f - 32.f) - 2.f;
    const bool c = 0.f > p[j] - 2.f;
    if (c) p[j] = -(p[j] - 2.f) + 2.f;
    f |= ((a ? 1u : 0u) | (b ? 2u : 0u) | (c ? 4u : 0u)) << (3 * j);
  }
  *fl = f;
}

__device__ __forceinline__ void bounce_sub_bwd(const Phys& P, unsigned fl, float* gp, float* gv) {
  for (int j = 1; j >= 0; --j) {
    const unsigned f = fl >> (3 * j);
    if (f & 4u) gp[j] = -gp[j];
    if (f & 1u) gp[j] = -gp[j];
    if (f & 2u) gv[j] = -gv[j];
    if (f & 1u) gv[j] = -gv[j];
  }
  gv[0] += P.h * gp[0];
  gv[1] += P.h * gp[1];
}

// --------------------------------------------------------------- gravity ----
__device__ __forceinline__ float clampf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

__device__ __forceinline__ void grav_force(const Phys& P, const float* p, float* F) {
  float vec[3][2], Fi[3][2];
  for (int c = 0; c < 2; ++c) {
    vec[0][c] = p[0 + c] - p[2 + c];
    vec[1][c] = p[2 + c] - p[4 + c];
    vec[2][c] = p[4 + c] - p[0 + c];
  }
  for (int i = 0; i < 3; ++i) {
    const float sq = vec[i][0] * vec[i][0] + vec[i][1] * vec[i][1];
    const float nrm = sqrtf(clampf(sq, 0.1f, 1e5f));
    const float cn = clampf(nrm, 1.f, 170.f);
    const float p3 = cn * cn * cn;
    Fi[i][0] = vec[i][0] / p3;
    Fi[i][1] = vec[i][1] / p3;
  }
  for (int c = 0; c < 2; ++c) {
    F[0 + c] = P.negA * (Fi[0][c] - Fi[2][c]);
    F[2 + c] = P.negA * (Fi[1][c] - Fi[0][c]);
    F[4 + c] = P.negA * (Fi[2][c] - Fi[1][c]);
  }
}

__device__ __forceinline__ void grav_sub(const Phys& P, float* p, float* v) {
  float F[6];
  grav_force(P, p, F);
  for (int i = 0; i < 6; ++i) v[i] = v[i] + P.h * F[i];
  for (int i = 0; i < 6; ++i) p[i] = p[i] + P.h * v[i];
}

__device__ __forceinline__ void grav_sub_bwd(const Phys& P, const float* p, float* gp, float* gv, float& gnegA) {
  for (int i = 0; i < 6; ++i) gv[i] += P.h * gp[i];
  float gF[6];
  for (int i = 0; i < 6; ++i) gF[i] = P.h * gv[i];
  // recompute force pieces
  float vec[3][2], Fi[3][2], cn[3], nrm[3], sq[3];
  for (int c = 0; c < 2; ++c) {
    vec[0][c] = p[0 + c] - p[2 + c];
    vec[1][c] = p[2 + c] - p[4 + c];
    vec[2][c] = p[4 + c] - p[0 + c];
  }
  for (int i = 0; i < 3; ++i) {
    sq[i] = vec[i][0] * vec[i][0] + vec[i][1] * vec[i][1];
    nrm[i] = sqrtf(clampf(sq[i], 0.1f, 1e5f));
    cn[i] = clampf(nrm[i], 1.f, 170.f);
    const float p3 = cn[i] * cn[i] * cn[i];
    Fi[i][0] = vec[i][0] / p3;
    Fi[i][1] = vec[i][1] / p3;
  }
  // F0 = negA (Fi0 - Fi2), F1 = negA (Fi1 - Fi0), F2 = negA (Fi2 - Fi1)
  float gFi[3][2];
  for (int c = 0; c < 2; ++c) {
    gnegA += (gF[0 + c] * (Fi[0][c] - Fi[2][c]) + gF[2 + c] * (Fi[1][c] - Fi[0][c]) +
                      gF[4 + c] * (Fi[2][c] - Fi[1][c]));
    const float a = P.negA * gF[0 + c], b = P.negA * gF[2 + c], d = P.negA * gF[4 + c];
    gFi[0][c] = a - b;
    gFi[1][c] = b - d;
    gFi[2][c] = d - a;
  }
  float gvec[3][2];
  for (int i = 0; i < 3; ++i) {
    const float p3 = cn[i] * cn[i] * cn[i];
    // Fi = vec / p3
    float gp3 = 0.f;
    for (int c = 0; c < 2; ++c) {
      gvec[i][c] = gFi[i][c] / p3;
      gp3 -= gFi[i][c] * vec[i][c] / (p3 * p3);
    }
    float gcn = gp3 * 3.f * cn[i] * cn[i];
    // cn = clamp(nrm, 1, 170): aten clamp' passes where lo <= x <= hi
    float gnrm = (nrm[i] >= 1.f && nrm[i] <= 170.f) ? gcn : 0.f;
    float csq = clampf(sq[i], 0.1f, 1e5f);
    float gcsq = gnrm / (2.f * sqrtf(csq));
    float gsq = (sq[i] >= 0.1f && sq[i] <= 1e5f) ? gcsq : 0.f;
    for (int c = 0; c < 2; ++c) gvec[i][c] += gsq * 2.f * vec[i][c];
  }
  for (int c = 0; c < 2; ++c) {
    gp[0 + c] += gvec[0][c] - gvec[2][c];
    gp[2 + c] += gvec[1][c] - gvec[0][c];
    gp[4 + c] += gvec[2][c] - gvec[1][c];
  }
}

struct PhysPtr {
  const float* dt;   // 0-dim fp32 parameter (requires_grad=False)
  const double* p0;  // k (spring) | g (gravity) | null
  const double* p1;  // equil (spring) | m (gravity) | null
};

template <int CELL>
__device__ __forceinline__ Phys load_phys(const PhysPtr& q) {
  Phys P;
  P.h = *q.dt / 5.0f;
  P.ek = 0.f;
  P.tee = 0.f;
  P.negA = 0.f;
  if (CELL == CELL_SPRING) {
    P.ek = (float)exp(*q.p0);
    P.tee = (float)(2.0 * exp(*q.p1));
  } else if (CELL == CELL_GRAVITY) {
    P.negA = (float)(-(exp(*q.p0) * exp(2.0 * *q.p1)));
  }
  return P;
}

template <int D, int CELL>
__device__ __forceinline__ void step_fwd(const Phys& P, float* p, float* v) {
  for (int s = 0; s < 5; ++s) {
    if (CELL == CELL_SPRING) spring_sub(P, p, v);
    else if (CELL == CELL_BOUNCE) { unsigned fl; bounce_sub(P, p, v, &fl); }
    else grav_sub(P, p, v);
  }
}

// pos0: [B] rows with stride pos0_ld ; vel0: [K][B][2] (object-major, the
// velocity MLP's output layout) or null (zeros); pvs: [B][1+R][2D]
template <int D, int CELL>
__global__ void rollout_fwd_k(const float* __restrict__ pos0, long long pos0_ld, const float* __restrict__ vel0,
                              PhysPtr Q, float* __restrict__ pvs, int B, int R) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const Phys P = load_phys<CELL>(Q);
  float p[D], v[D];
  for (int d = 0; d < D; ++d) {
    p[d] = pos0[(long long)b * pos0_ld + d];
    v[d] = vel0 ? vel0[((long long)(d >> 1) * B + b) * 2 + (d & 1)] : 0.f;
  }
  float* o = pvs + (long long)b * (R + 1) * 2 * D;
  for (int d = 0; d < D; ++d) {
    o[d] = p[d];
    o[D + d] = v[d];
  }
  for (int t = 1; t <= R; ++t) {
    step_fwd<D, CELL>(P, p, v);
    for (int d = 0; d < D; ++d) {
      o[t * 2 * D + d] = p[d];
      o[t * 2 * D + D + d] = v[d];
    }
  }
}

// dpos_roll: [B][R][D] adjoint of the rolled-out positions (decoder input), may be null
// dpvs: [B][1+R][2D] adjoint of pos_vel_seq, may be null
// out: dpos0 [B][D], dvel0 [K][B][2] (same layout as vel0), part [gridDim][2] fp64
template <int D, int CELL>
__global__ void __launch_bounds__(256)
rollout_bwd_k(const float* __restrict__ pvs, const float* __restrict__ dpos_roll, const float* __restrict__ dpvs,
              PhysPtr Q, float* __restrict__ dpos0, float* __restrict__ dvel0, double* __restrict__ part, int B, int R) {
  __shared__ double red[4][2];
  const Phys P = load_phys<CELL>(Q);
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  double g0 = 0.0, g1 = 0.0;
  if (b < B) {
    float gp[D], gv[D];
    for (int d = 0; d < D; ++d) gp[d] = gv[d] = 0.f;
    const float* st = pvs + (long long)b * (R + 1) * 2 * D;
    // the serial reverse sweep would wait one global-load latency per step for
    // its inputs: they are prefetched one step ahead, behind the substep math
    float nd[D], ns[2 * D];
    for (int d = 0; d < D; ++d) nd[d] = dpos_roll ? dpos_roll[((long long)b * R + (R - 1)) * D + d] : 0.f;
    for (int d = 0; d < 2 * D; ++d) ns[d] = st[(R - 1) * 2 * D + d];
    for (int t = R; t >= 1; --t) {
      float cd[D], cs[2 * D];
      for (int d = 0; d < D; ++d) cd[d] = nd[d];
      for (int d = 0; d < 2 * D; ++d) cs[d] = ns[d];
      if (t > 1) {
        for (int d = 0; d < D; ++d) nd[d] = dpos_roll ? dpos_roll[((long long)b * R + (t - 2)) * D + d] : 0.f;
        for (int d = 0; d < 2 * D; ++d) ns[d] = st[(t - 2) * 2 * D + d];
      }
      for (int d = 0; d < D; ++d) gp[d] += cd[d];
      if (dpvs)
        for (int d = 0; d < D; ++d) {
          gp[d] += dpvs[((long long)b * (R + 1) + t) * 2 * D + d];
          gv[d] += dpvs[((long long)b * (R + 1) + t) * 2 * D + D + d];
        }
      // recompute the 5 substep input states of step t (from state t-1)
      float ps[5][D], vs[5][D];
      unsigned fl[5];
      float p[D], v[D];
      for (int d = 0; d < D; ++d) {
        p[d] = cs[d];
        v[d] = cs[D + d];
      }
#pragma unroll
      for (int s = 0; s < 5; ++s) {
        for (int d = 0; d < D; ++d) {
          ps[s][d] = p[d];
          vs[s][d] = v[d];
        }
        if (CELL == CELL_SPRING) spring_sub(P, p, v);
        else if (CELL == CELL_BOUNCE) bounce_sub(P, p, v, &fl[s]);
        else grav_sub(P, p, v);
      }
      float s0 = 0.f, s1 = 0.f;   // this step's parameter adjoints
#pragma unroll
      for (int s = 4; s >= 0; --s) {
        if (CELL == CELL_SPRING) spring_sub_bwd(P, ps[s], vs[s], gp, gv, s0, s1);
        else if (CELL == CELL_BOUNCE) bounce_sub_bwd(P, fl[s], gp, gv);
        else grav_sub_bwd(P, ps[s], gp, gv, s0);
      }
      g0 += (double)s0;
      g1 += (double)s1;
    }
    if (dpvs)
      for (int d = 0; d < D; ++d) {
        gp[d] += dpvs[((long long)b * (R + 1)) * 2 * D + d];
        gv[d] += dpvs[((long long)b * (R + 1)) * 2 * D + D + d];
      }
    for (int d = 0; d < D; ++d) {
      dpos0[(long long)b * D + d] = gp[d];
      if (dvel0) dvel0[((long long)(d >> 1) * B + b) * 2 + (d & 1)] = gv[d];
    }
  }
  g0 = wave_sum_d(g0);
  g1 = wave_sum_d(g1);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) {
    red[wv][0] = g0;
    red[wv][1] = g1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, c = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
      a += red[w][0];
      c += red[w][1];
    }
    part[blockIdx.x * 2 + 0] = a;
    part[blockIdx.x * 2 + 1] = c;
  }
}

// ------------------------------------------------ spring adjoint as a scan ----
// The adjoint of the spring rollout is a linear recurrence in time: with x_t
// the adjoint of the moving state (p0, p1, v0, v1) entering step t's backward,
//   x_t = b_t + M_{t+1} x_{t+1},  x_{R+1} = 0,      a_0 = M_1 x_1 + b_0,
// where M_t is the transposed Jacobian of step t's 5 substeps (it depends only
// on the stored state t-1) and b_t the injected adjoints of step t's outputs.
// The physics-parameter adjoints of step t are linear forms u_t, w_t of x_t.
// One wave per sequence, lane t-1 owns step t: every lane recomputes its
// step's substeps and builds M_t, u_t, w_t by pushing the 4 basis vectors
// through the substep adjoints (parallel over the R steps), then a reverse
// Hillis-Steele scan over the lanes composes (M, b) pairs: log2(64) rounds of
// a 4x4 product instead of R x 5 dependent substep adjoints on one lane.
// Columns 2, 3 (object 1 under the split-size-1 quirk Q3) never move: their
// adjoints are plain sums of the injections.
__global__ void __launch_bounds__(256)
rollout_bwd_spring_scan_k(const float* __restrict__ pvs, const float* __restrict__ dpos_roll,
                          const float* __restrict__ dpvs, PhysPtr Q, float* __restrict__ dpos0,
                          float* __restrict__ dvel0, double* __restrict__ part, int B, int R) {
  constexpr int D = 4;
  __shared__ double red[4][2];
  const Phys P = load_phys<CELL_SPRING>(Q);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int b = blockIdx.x * 4 + wv;   // sequence of this wave
  double g0 = 0.0, g1 = 0.0;
  if (b < B) {                          // wave-uniform
    const int t = lane + 1;             // this lane's step
    const bool live = t <= R;
    const float* st = pvs + (long long)b * (R + 1) * 2 * D;
    // ---- M_t (column j = adjoint of basis e_j through the 5 substeps), u_t, w_t
    float M[4][4] = {}, u[4] = {}, wq[4] = {};
    if (live) {
      float ps[5][2], vs[5][2];
      float p[D], v[D];
      for (int d = 0; d < D; ++d) {
        p[d] = st[(t - 1) * 2 * D + d];
        v[d] = st[(t - 1) * 2 * D + D + d];
      }
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        ps[q][0] = p[0];
        ps[q][1] = p[1];
        vs[q][0] = v[0];
        vs[q][1] = v[1];
        spring_sub(P, p, v);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float gp[D] = {0.f, 0.f, 0.f, 0.f}, gv[D] = {0.f, 0.f, 0.f, 0.f};
        if (j < 2) gp[j] = 1.f;
        else gv[j - 2] = 1.f;
        float a = 0.f, c = 0.f;
#pragma unroll
        for (int q = 4; q >= 0; --q) {
          const float pq[D] = {ps[q][0], ps[q][1], 0.f, 0.f}, vq[D] = {vs[q][0], vs[q][1], 0.f, 0.f};
          spring_sub_bwd(P, pq, vq, gp, gv, a, c);
        }
        M[0][j] = gp[0];
        M[1][j] = gp[1];
        M[2][j] = gv[0];
        M[3][j] = gv[1];
        u[j] = a;
        wq[j] = c;
      }
    }
    // ---- injections b_t (t = 1..R) of the moving components; columns 2, 3 summed
    float bx[4] = {0.f, 0.f, 0.f, 0.f}, fixp[2] = {0.f, 0.f}, fixv[2] = {0.f, 0.f};
    if (live) {
      if (dpos_roll) {
        const float* q = dpos_roll + ((long long)b * R + (t - 1)) * D;
        bx[0] += q[0];
        bx[1] += q[1];
        fixp[0] += q[2];
        fixp[1] += q[3];
      }
      if (dpvs) {
        const float* q = dpvs + ((long long)b * (R + 1) + t) * 2 * D;
        bx[0] += q[0];
        bx[1] += q[1];
        bx[2] += q[D];
        bx[3] += q[D + 1];
        fixp[0] += q[2];
        fixp[1] += q[3];
        fixv[0] += q[D + 2];
        fixv[1] += q[D + 3];
      }
    }
    // ---- reverse scan: element t = (A, B) with x_t = B + A x_{t+1}; A_t = M_{t+1}
    float A[4][4], Bv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      Bv[r] = bx[r];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float m = __shfl_down(M[r][c], 1, 64);
        A[r][c] = t + 1 <= R ? m : 0.f;
      }
    }
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
      float A2[4][4], B2[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        B2[r] = __shfl_down(Bv[r], k, 64);
#pragma unroll
        for (int c = 0; c < 4; ++c) A2[r][c] = __shfl_down(A[r][c], k, 64);
      }
      if (lane + k < 64) {   // (A, B) <- (A A2, B + A B2): the segment [t .. t + 2k)
        float An[4][4], Bn[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          Bn[r] = Bv[r];
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            Bn[r] += A[r][c] * B2[c];
            float acc = 0.f;
#pragma unroll
            for (int m = 0; m < 4; ++m) acc += A[r][m] * A2[m][c];
            An[r][c] = acc;
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          Bv[r] = Bn[r];
#pragma unroll
          for (int c = 0; c < 4; ++c) A[r][c] = An[r][c];
        }
      }
    }
    // lane t-1 now holds x_t = Bv (the suffix reaches past R, where x = 0)
    const float s0 = live ? u[0] * Bv[0] + u[1] * Bv[1] + u[2] * Bv[2] + u[3] * Bv[3] : 0.f;
    const float s1 = live ? wq[0] * Bv[0] + wq[1] * Bv[1] + wq[2] * Bv[2] + wq[3] * Bv[3] : 0.f;
    g0 = (double)s0;
    g1 = (double)s1;
    const float fp0 = wave_sum(fixp[0]), fp1 = wave_sum(fixp[1]), fv0 = wave_sum(fixv[0]), fv1 = wave_sum(fixv[1]);
    if (lane == 0) {   // a_0 = M_1 x_1 + b_0
      float a0[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) a0[r] = M[r][0] * Bv[0] + M[r][1] * Bv[1] + M[r][2] * Bv[2] + M[r][3] * Bv[3];
      float gp[D] = {a0[0], a0[1], fp0, fp1}, gv[D] = {a0[2], a0[3], fv0, fv1};
      if (dpvs) {
        const float* q = dpvs + (long long)b * (R + 1) * 2 * D;
        for (int d = 0; d < D; ++d) {
          gp[d] += q[d];
          gv[d] += q[D + d];
        }
      }
      for (int d = 0; d < D; ++d) {
        dpos0[(long long)b * D + d] = gp[d];
        if (dvel0) dvel0[((long long)(d >> 1) * B + b) * 2 + (d & 1)] = gv[d];
      }
    }
  }
  g0 = wave_sum_d(g0);
  g1 = wave_sum_d(g1);
  if (lane == 0) {
    red[wv][0] = g0;
    red[wv][1] = g1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, c = 0.0;
    for (int w = 0; w < 4; ++w) {
      a += red[w][0];
      c += red[w][1];
    }
    part[blockIdx.x * 2 + 0] = a;
    part[blockIdx.x * 2 + 1] = c;
  }
}

// finalize physics-parameter grads (fp64): spring: dk = sum(gek)*ek, dequil =
// sum(gtee)*tee ; gravity: dg = sum(gnegA) * negA.  out[0..1] (+)= ...
__global__ void rollout_param_final_k(const double* __restrict__ part, int nblk, int cell, PhysPtr Q,
                                      double* __restrict__ g0, double* __restrict__ g1, int accumulate) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const double ek = cell == CELL_SPRING ? exp(*Q.p0) : 0.0;
  const double tee = cell == CELL_SPRING ? 2.0 * exp(*Q.p1) : 0.0;
  const double negA = cell == CELL_GRAVITY ? -(exp(*Q.p0) * exp(2.0 * *Q.p1)) : 0.0;
  double a = 0.0, c = 0.0;
  for (int i = 0; i < nblk; ++i) {
    a += part[2 * i];
    c += part[2 * i + 1];
  }
  if (cell == CELL_SPRING) {
    // ek = exp(k) -> d/dk = ek ; tee = 2 exp(equil) -> d/dequil = tee
    const double dk = (double)(float)a * ek, de = (double)(float)c * tee;
    if (g0) *g0 = accumulate ? *g0 + dk : dk;
    if (g1) *g1 = accumulate ? *g1 + de : de;
  } else if (cell == CELL_GRAVITY) {
    // negA = -exp(g) exp(2m) -> d/dg = negA
    const double dg = (double)(float)a * negA;
    if (g0) *g0 = accumulate ? *g0 + dg : dg;
  }
}

template <int D, int CELL>
static int launch_fwd(const float* pos0, long long ld, const float* vel0, PhysPtr P, float* pvs, int B, int R,
                      hipStream_t st) {
  hipLaunchKernelGGL((rollout_fwd_k<D, CELL>), dim3(cdiv(B, 64)), dim3(64), 0, st, pos0, ld, vel0, P, pvs, B, R);
  PAIG_CHECK_LAUNCH();
  return 0;
}

template <int D, int CELL>
static int launch_bwd(const float* pvs, const float* dpr, const float* dpvs, PhysPtr P, float* dpos0, float* dvel0,
                      double* part, int B, int R, hipStream_t st) {
  hipLaunchKernelGGL((rollout_bwd_k<D, CELL>), dim3(cdiv(B, 64)), dim3(64), 0, st, pvs, dpr, dpvs, P, dpos0, dvel0,
                     part, B, R);
  PAIG_CHECK_LAUNCH();
  return 0;
}

}  // namespace

extern "C" {

// cell: 0 spring (params k, equil), 1 bouncing (none), 2 gravity (params g, m).
// dt: 0-dim fp32 device param; p0/p1: 0-dim fp64 device params (k, equil)
// or (g, m); null for bouncing.  Nothing is read back to the host.
int paig_rollout_fwd(int cell, const float* pos0, long long pos0_ld, const float* vel0, const float* dt,
                     const double* p0, const double* p1, float* pvs, int B, int D, int R, void* stream) {
  if (B <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  PAIG_REQUIRE(cell == CELL_BOUNCE || (p0 && p1), "rollout: physics params required");
  PhysPtr P{dt, p0, p1};
  if (cell == CELL_SPRING && D == 4) return launch_fwd<4, CELL_SPRING>(pos0, pos0_ld, vel0, P, pvs, B, R, st);
  if (cell == CELL_BOUNCE && D == 4) return launch_fwd<4, CELL_BOUNCE>(pos0, pos0_ld, vel0, P, pvs, B, R, st);
  if (cell == CELL_GRAVITY && D == 6) return launch_fwd<6, CELL_GRAVITY>(pos0, pos0_ld, vel0, P, pvs, B, R, st);
  paig_set_error("rollout: unsupported cell %d with D=%d", cell, D);
  return PAIG_E_UNSUPPORTED;
}

// partial-slab rows of paig_rollout_bwd: one per block (64 sequences per
// block serially, or 4 per block for the spring scan: the larger count)
int paig_rollout_bwd_blocks(int B) { return cdiv(B, 4); }

int paig_rollout_bwd(int cell, const float* pvs, const float* dpos_roll, const float* dpvs, const float* dt,
                     const double* p0, const double* p1, float* dpos0, float* dvel0, double* part, double* gparam0,
                     double* gparam1, int accumulate, int B, int D, int R, void* stream) {
  if (B <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  PAIG_REQUIRE(cell == CELL_BOUNCE || (p0 && p1), "rollout: physics params required");
  PhysPtr P{dt, p0, p1};
  int rc, nblk = cdiv(B, 64);
  if (cell == CELL_SPRING && D == 4 && R <= 64) {   // one wave per sequence, a lane per step
    nblk = cdiv(B, 4);
    hipLaunchKernelGGL(rollout_bwd_spring_scan_k, dim3(nblk), dim3(256), 0, st, pvs, dpos_roll, dpvs, P, dpos0, dvel0,
                       part, B, R);
    PAIG_CHECK_LAUNCH();
    rc = 0;
  } else if (cell == CELL_SPRING && D == 4) rc = launch_bwd<4, CELL_SPRING>(pvs, dpos_roll, dpvs, P, dpos0, dvel0, part, B, R, st);
  else if (cell == CELL_BOUNCE && D == 4) rc = launch_bwd<4, CELL_BOUNCE>(pvs, dpos_roll, dpvs, P, dpos0, dvel0, part, B, R, st);
  else if (cell == CELL_GRAVITY && D == 6) rc = launch_bwd<6, CELL_GRAVITY>(pvs, dpos_roll, dpvs, P, dpos0, dvel0, part, B, R, st);
  else {
    paig_set_error("rollout: unsupported cell %d with D=%d", cell, D);
    return PAIG_E_UNSUPPORTED;
  }
  if (rc) return rc;
  if (cell != CELL_BOUNCE) {
    hipLaunchKernelGGL(rollout_param_final_k, dim3(1), dim3(64), 0, st, part, nblk, cell, P, gparam0, gparam1,
                       accumulate);
    PAIG_CHECK_LAUNCH();
  }
  return 0;
}

}  // extern "C"
