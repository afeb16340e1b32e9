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

#include "rollout_cells.h"

// pos0: [B] rows with stride pos0_ld ; vel0: [K][B][2] (object-major, the
// velocity MLP's output layout) or null (zeros); pvs: [B][1+R][2D]
template <int D, int CELL>
__global__ void rollout_fwd_k(const float* __restrict__ pos0, long long pos0_ld, const float* __restrict__ vel0,
                              PhysPtr Q, float* __restrict__ pvs, int B, int R) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  rollout_fwd_seq<D, CELL>(pos0, pos0_ld, vel0, Q, pvs, B, R, b);
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
