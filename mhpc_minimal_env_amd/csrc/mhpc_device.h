// Device-side helpers shared by the solve kernels: cost weights, references, reduced
// barrier, foothold planner.  Every helper restates reference code cited at its definition.
#pragma once
#include <hip/hip_runtime.h>

#include "mhpc_model.h"
#include "mhpc_solver.h"

namespace MHPC_NS {

constexpr real PI = real(3.141592653589793238);  // MHPC_CPPTypes.h:18

// Cost weights and constraint parameters live in SolveParams::cw (mhpc_set_cost_weights /
// mhpc_set_constraint_params; defaults MHPCCost.cpp:24-75, MHPCConstraints.cpp:14-88).
// terminal WB state references (ReferenceGen.cpp:45-52), velocity entry filled at run time
static __constant__ real cXtermWB[4][14] = {
    {0, -real(0.1432), -PI / 25, real(0.35) * PI, -real(0.65) * PI, real(0.35) * PI, -real(0.6) * PI, 0, 1, 0, 0, 0, 0, 0},
    {0, -real(0.1418), PI / 35, real(0.2) * PI, -real(0.58) * PI, real(0.25) * PI, -real(0.7) * PI, 0, -1, 0, 0, 0, 0, 0},
    {0, -real(0.1325), -PI / 40, real(0.33) * PI, -real(0.48) * PI, real(0.33) * PI, -real(0.75) * PI, 0, 1, 0, 0, 0, 0, 0},
    {0, -real(0.1490), -PI / 25, real(0.35) * PI, -real(0.7) * PI, real(0.25) * PI, -real(0.60) * PI, 0, -1, 0, 0, 0, 0, 0}};
static __constant__ real cQjointBias[4] = {real(0.3) * PI, -real(0.7) * PI, real(0.3) * PI, -real(0.7) * PI};
constexpr real kGRF = real(8.252) * real(9.81);  // ReferenceGen.cpp:27

static __device__ __forceinline__ real* traj_ptr(const SolveParams& sp, const DevBufs& d, int b,
                                            int slot, int kk) {
  return d.traj + (((size_t)b * sp.nslot + slot) * sp.NK + kk) * KS;
}

static __device__ __forceinline__ int ntc_of(int mode, bool wb) { return wb && (mode == 2 || mode == 4); }

// ---- layout groups ----------------------------------------------------------------------
// A launch over the batch enumerates its blocks group by group: group g (problems
// gidx[go[g] .. go[g+1]), layout g) takes ceil(n_g / per) blocks of `per` problems, so every
// wave of a block runs one layout (uniform control flow, the layout in scalar registers).
struct GrpBlk {
  int g;       // layout group (-1: block past the last group)
  int p0, p1;  // the block's first gidx position and the end of its group's positions
};
static __device__ __forceinline__ GrpBlk block_group(const SolveParams& sp, int blk, int per) {
  int start = 0;
  for (int g = 0; g < sp.ngrp; ++g) {
    const int n = sp.go[g + 1] - sp.go[g], nb = (n + per - 1) / per;
    if (blk < start + nb) return {g, sp.go[g] + (blk - start) * per, sp.go[g + 1]};
    start += nb;
  }
  return {-1, 0, 0};
}
// The same for launches of `per_item` items per problem (e.g. the partials' knots) in blocks
// of `nt` lanes: group g takes ceil(n_g * items_g / nt) blocks; *t0 = the block's first item
// of the group (problem position go[g] + item / items_g).
// (items == nullptr: n_items for every group)
static __device__ __forceinline__ int block_group_items(const SolveParams& sp, const int* items,
                                                         int n_items, int blk, int nt, long* t0) {
  int start = 0;
  for (int g = 0; g < sp.ngrp; ++g) {
    const long n = (long)(sp.go[g + 1] - sp.go[g]) * (items ? items[g] : n_items);
    const int nb = (int)((n + nt - 1) / nt);
    if (blk < start + nb) {
      *t0 = (long)(blk - start) * nt;
      return g;
    }
    start += nb;
  }
  return -1;
}
// Problem index at gidx position pos.
static __device__ __forceinline__ int prob_at(const SolveParams& sp, const DevBufs& d, int pos) {
  return sp.ident ? pos : d.gidx[pos];
}
// Layout g, read through the constant address space: the table never changes during a launch,
// so every field a wave-uniform index selects is a scalar load (s_load), as a parameter-block
// field would be, never a vector load plus readfirstlane.
typedef const __attribute__((address_space(4))) Layout CLayout;
static __device__ __forceinline__ const Layout& layout_of(const DevBufs& d, int g) {
  return *(const Layout*)((CLayout*)d.lay + g);
}

// Natural log of a positive argument (the barrier's g > delta > 0 and delta itself).  fp64:
// the fdlibm algorithm (e_log.c: x = 2^k (1 + f) with sqrt(2)/2 <= 1 + f < sqrt(2),
// s = f / (2 + f), a degree-14 odd polynomial in s), < 1 ulp -- about a third of the
// instructions of the library log, whose extra work covers denormal scaling and special
// values this path never sees.  The line search evaluates up to 11 of these per WB knot
// and candidate while the ReB barrier is active.
static __device__ __forceinline__ real log_pos(real x) {
  MHPC_NO_FMA_F32
#ifdef MHPC_FP32
  return logf(x);
#else
  int k;
  double m = frexp(x, &k);  // x = m 2^k, m in [0.5, 1)
  const bool lo = m < 0.70710678118654752440;
  m = lo ? m + m : m;
  k = lo ? k - 1 : k;
  const double f = m - 1.0;
  const double s = f / (2.0 + f);
  const double z = s * s, w = z * z;
  const double t1 = w * (3.999999999940941908e-01 + w * (2.222219843214978396e-01 +
                                                         w * 1.531383769920937332e-01));
  const double t2 = z * (6.666666666666735130e-01 +
                         w * (2.857142874366239149e-01 +
                              w * (1.818357216161805012e-01 + w * 1.479819860511658591e-01)));
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  const double dk = (double)k;
  return dk * 6.93147180369123816490e-01 -
         ((hfsq - (s * (hfsq + R) + dk * 1.90821492927058770002e-10)) - f);
#endif
}

// ---- reduced barrier (SinglePhase.cpp:298-317), k = 2 ---------------------------------
// The reference's pow() calls with integer exponents are evaluated exactly as products:
// pow(t, 2) = t*t (the correctly rounded square), pow(t, 1) = t, pow(t, 0) = 1 (also for
// NaN, as pow defines), pow(g, -2) = 1/(g*g) (within 1 ulp of the correctly rounded value).
// One log per constraint (of g or of delta, whichever side the lane takes) outside the branch,
// so a wave whose lanes split over the two sides evaluates one log, not both; the relaxed
// side's extra work stays behind a branch that waves far from the constraint skip.  Each lane
// computes exactly the operations of its side.
static __device__ __forceinline__ void reduced_barrier(real g, real delta, real* B, real* Bz,
                                                real* Bzz) {
  MHPC_NO_FMA_F32
  const bool in = g > delta;
  const real lg = log_pos(in ? g : delta);
  if (in) {
    *B = -lg;
    *Bz = -1.0 / g;
    *Bzz = 1.0 / (g * g);
  } else {
    const real t = (g - 2 * delta) / ((2 - 1) * delta);
    *B = (real)(2 - 1) / 2 * (t * t - 1) - lg;
    *Bz = t / delta;
    *Bzz = 1.0;
  }
}

// Running cost value incl. the ReB barrier of WB phases (CostBase.cpp:4-16,
// SinglePhase.cpp:219-249 in CALC_DYNAMICS_ONLY), reference of knot kk built in registers.
static __device__ real wb_running_cost(const SolveParams& sp, int mode, real dt, real pos,
                                  const real* x, const real* u, const real* y, bool reb,
                                  real delta, real eps_tq, real eps_grf) {
  MHPC_NO_FMA_COST
  const int m = mode - 1;
  real rx[14] = {pos, sp.height, 0, cQjointBias[0], cQjointBias[1], cQjointBias[2],
                   cQjointBias[3], sp.vel, 0, 0, 0, 0, 0, 0};
  const real ry[4] = {0, kGRF, 0, kGRF};
  real l = 0, t = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i) { const real e = x[i] - rx[i]; l += e * sp.cw.wQ[m][i] * e; }
#pragma unroll
  for (int i = 0; i < 4; ++i) { const real e = u[i]; t += e * sp.cw.wR[m][i] * e; }
  l += t;
  t = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) { const real e = y[i] - ry[i]; t += e * sp.cw.wS[m][i] * e; }
  l += t;
  l = l * dt;
  if (reb) {
    real B, Bz, Bzz;
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // torque limits tq_lim -/+ u
      const real g = (i < 4 ? -u[i] : u[i - 4]) + sp.cw.tq_lim;
      reduced_barrier(g, delta, &B, &Bz, &Bzz);
      l += eps_tq * B * dt;
    }
    // joint limits carry eps_ReB = 0 (MHPCConstraints.cpp:64-84): contribution 0 * B * dt
    if (mode == 1 || mode == 3) {  // GRF: Fz >= 0, mu Fz -/+ Fx >= 0
      const int o = mode == 1 ? 2 : 0;
      const real mu = sp.cw.mu;
      const real gs[3] = {y[o + 1], -y[o] + mu * y[o + 1], y[o] + mu * y[o + 1]};
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        reduced_barrier(gs[i], delta, &B, &Bz, &Bzz);
        l += eps_grf * B * dt;
      }
    }
  }
  return l;
}

static __device__ real fb_running_cost(const SolveParams& sp, int mode, real dt, real pos,
                                  const real* x, const real* u) {
  MHPC_NO_FMA_COST
  const int m = mode - 1;
  const real rx[6] = {pos, sp.height, 0, sp.vel, 0, 0};
  const real ru[4] = {0, kGRF, 0, kGRF};
  real l = 0, t = 0;
#pragma unroll
  for (int i = 0; i < 6; ++i) { const real e = x[i] - rx[i]; l += e * sp.cw.fQ[m][i] * e; }
#pragma unroll
  for (int i = 0; i < 4; ++i) { const real e = u[i] - ru[i]; t += e * sp.cw.fR[m][i] * e; }
  l += t;
  l += real(0.0);  // S = 0 for the floating base (y = 0)
  return l * dt;
}

// Derivatives of a WB running cost w.r.t. u and the stance force (CostBase.cpp:19-34 and
// the CALC_PARTIALS_ONLY branch of SinglePhase.cpp:219-249; joint limits carry eps_ReB = 0
// and contribute exact zeros).  out = lu[4], luu[4] (diagonal), ly[2], lyy[4] where ly/lyy
// are the entries of the stance foot's force slots (zero in flight).
static __device__ void wb_cost_uy_derivs(const SolveParams& sp, int mode, real dt, const real* u,
                                         const real* y, bool reb, real delta, real eps_tq,
                                         real eps_grf, real* out) {
  const int m = mode - 1;
  const real tq = sp.cw.tq_lim, mu = sp.cw.mu;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    real lu = (2 * dt * sp.cw.wR[m][c]) * (u[c] - real(0.0));
    real luu = 2 * dt * sp.cw.wR[m][c];
    if (reb) {
      real B, Bz, Bzz;
      // constraint c: g = -u_c + tq (gu = -1); constraint 4 + c: g = u_c + tq (gu = +1)
      reduced_barrier(-real(1.0) * u[c] + tq, delta, &B, &Bz, &Bzz);
      lu += eps_tq * Bz * -real(1.0) * dt;
      luu += eps_tq * (-real(1.0) * Bzz * -real(1.0)) * dt;
      reduced_barrier(real(1.0) * u[c] + tq, delta, &B, &Bz, &Bzz);
      lu += eps_tq * Bz * real(1.0) * dt;
      luu += eps_tq * (real(1.0) * Bzz * real(1.0)) * dt;
    }
    out[c] = lu;
    out[4 + c] = luu;
  }
  out[8] = out[9] = out[10] = out[11] = out[12] = out[13] = real(0.0);
  if (mode == 1 || mode == 3) {
    const int o = mode == 1 ? 2 : 0;
    const real fx = mode == 1 ? y[2] : y[0], fz = mode == 1 ? y[3] : y[1];
    const real s0 = sp.cw.wS[m][o], s1 = sp.cw.wS[m][o + 1];
    real ly0 = (2 * dt * s0) * (fx - real(0.0));
    real ly1 = (2 * dt * s1) * (fz - kGRF);
    real l00 = 2 * dt * s0, l01 = real(0.0), l10 = real(0.0), l11 = 2 * dt * s1;
    if (reb) {
      const real rows[3][2] = {{0, 1}, {-1, mu}, {1, mu}};  // coefficients on (Fx, Fz)
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        real B, Bz, Bzz;
        reduced_barrier(rows[i][0] * fx + rows[i][1] * fz + 0, delta, &B, &Bz, &Bzz);
        ly0 += eps_grf * Bz * rows[i][0] * dt;
        ly1 += eps_grf * Bz * rows[i][1] * dt;
        l00 += eps_grf * (rows[i][0] * Bzz * rows[i][0]) * dt;
        l01 += eps_grf * (rows[i][0] * Bzz * rows[i][1]) * dt;
        l10 += eps_grf * (rows[i][1] * Bzz * rows[i][0]) * dt;
        l11 += eps_grf * (rows[i][1] * Bzz * rows[i][1]) * dt;
      }
    }
    out[8] = ly0; out[9] = ly1;
    out[10] = l00; out[11] = l01; out[12] = l10; out[13] = l11;
  }
}

static __device__ void wb_term_ref(const SolveParams& sp, int mode, real pos, real* rx) {
  MHPC_NO_FMA_F32
#pragma unroll
  for (int i = 0; i < 14; ++i) rx[i] = cXtermWB[mode - 1][i];
  rx[7] = sp.vel;
  rx[0] = pos;
}

static __device__ void fb_term_ref(const SolveParams& sp, real pos, real* rx) {
  MHPC_NO_FMA_F32
  rx[0] = pos; rx[1] = sp.height; rx[2] = 0; rx[3] = sp.vel; rx[4] = 0; rx[5] = 0;
}

// FootholdPlanner::get_foothold_location (FootholdPlan.h:26-50), velcmd 1.5 / ground
// -0.404 hard-coded by the reference (MHPCLocomotion.cpp:25).
static __device__ void plan_foothold(const real* x0, real stance_time, int mode, real* f) {
  MHPC_NO_FMA_F32
  f[0] = f[1] = f[2] = f[3] = 0;
  if (mode == 1) {
    f[2] = (cos(x0[2]) * (-real(0.19)) + x0[0]) + real(1.5) * stance_time / 2;
    f[3] = -real(0.404);
  } else if (mode == 3) {
    f[0] = (cos(x0[2]) * real(0.19) + x0[0]) + real(1.5) * stance_time / 2;
    f[1] = -real(0.404);
  }
}


}  // namespace MHPC_NS
