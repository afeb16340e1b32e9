// Physics cells of the differentiable rollout (nn/network/cells.py), shared
// by rollout.hip (the rollout and its adjoint) and decoder.hip (the rollout
// launched beside the reconstruction decode, paig_decoder_fwd_rollout).
// Included inside each translation unit's anonymous namespace.
#pragma once

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

// one sequence's rollout (thread b): pos0: [B] rows with stride pos0_ld;
// vel0: [K][B][2] (object-major, the velocity MLP's output layout) or null
// (zeros); pvs: [B][1+R][2D]
template <int D, int CELL>
__device__ __forceinline__ void rollout_fwd_seq(const float* __restrict__ pos0, long long pos0_ld,
                                                const float* __restrict__ vel0, const PhysPtr& Q, float* __restrict__ pvs,
                                                int B, int R, int b) {
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
