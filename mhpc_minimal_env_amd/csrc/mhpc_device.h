// Device-side helpers shared by the solve kernels: cost weights, references, reduced
// barrier, foothold planner.  Every helper restates reference code cited at its definition.
#pragma once
#include <hip/hip_runtime.h>

#include "mhpc_model.h"
#include "mhpc_solver.h"

namespace mhpc {

constexpr double PI = 3.141592653589793238;  // MHPC_CPPTypes.h:18

// ---- cost weights (MHPCCost.cpp:24-75) ------------------------------------------------
static __constant__ double cQwb[14] = {0.01 * 0, 0.01 * 10, 0.01 * 5, 0.01 * 4, 0.01 * 4, 0.01 * 4,
                                0.01 * 4, 0.01 * 2, 0.01 * 1, 0.01 * .01, 0.01 * 6, 0.01 * 6,
                                0.01 * 6, 0.01 * 6};
static __constant__ double cQfwb[4][14] = {
    {100 * 0., 100 * 20., 100 * 8., 100 * 3., 100 * 3., 100 * 3., 100 * 3., 100 * 3., 100 * 2.,
     100 * 0.01, 100 * 5., 100 * 5., 100 * 0.01, 100 * 0.01},
    {100 * 0., 100 * 20., 100 * 8., 100 * 3., 100 * 3., 100 * 3., 100 * 3., 100 * 3., 100 * 2.,
     100 * 0.01, 100 * 5., 100 * 5., 100 * 5., 100 * 5.},
    {100 * 0., 100 * 20., 100 * 8., 100 * 3., 100 * 3., 100 * 3., 100 * 3., 100 * 3., 100 * 2.,
     100 * 0.01, 100 * 0.01, 100 * 0.01, 100 * 5., 100 * 5.},
    {100 * 0., 100 * 20., 100 * 8., 100 * 3., 100 * 3., 100 * 3., 100 * 3., 100 * 3., 100 * 2.,
     100 * 0.01, 100 * 5., 100 * 5., 100 * 5., 100 * 5.}};
static __constant__ double cRwb[4][4] = {{0.5 * 5, 0.5 * 5, 0.5 * 1, 0.5 * 1},
                                  {0.5 * 1, 0.5 * 1, 0.5 * 1, 0.5 * 1},
                                  {0.5 * 1, 0.5 * 1, 0.5 * 5, 0.5 * 5},
                                  {0.5 * 1, 0.5 * 1, 0.5 * 1, 0.5 * 1}};
// s[3] is uninitialised in the reference (MHPCCost.cpp:43 fills s[0..2]); zero here, as in
// the oracle.  It can only offset the value of WB mode-4 running costs (y = 0 in flight).
static __constant__ double cSwb[4][4] = {{0, 0, 0.3, 0.3}, {0, 0, 0, 0}, {0.15, 0.15, 0, 0}, {0, 0, 0, 0}};
static __constant__ double cQfb[6] = {0.01 * 0, 0.01 * 10, 0.01 * 5, 0.01 * 2, 0.01 * 1, 0.01 * 0.01};
static __constant__ double cQffb[6] = {100 * 1., 100 * 20., 100 * 8., 100 * 3., 100 * 1., 100 * 0.01};
static __constant__ double cRfb[4][4] = {{0, 0, 0.01, 0.01}, {0, 0, 0, 0}, {0.01, 0.01, 0, 0}, {0, 0, 0, 0}};
// terminal WB state references (ReferenceGen.cpp:45-52), velocity entry filled at run time
static __constant__ double cXtermWB[4][14] = {
    {0, -0.1432, -PI / 25, 0.35 * PI, -0.65 * PI, 0.35 * PI, -0.6 * PI, 0, 1, 0, 0, 0, 0, 0},
    {0, -0.1418, PI / 35, 0.2 * PI, -0.58 * PI, 0.25 * PI, -0.7 * PI, 0, -1, 0, 0, 0, 0, 0},
    {0, -0.1325, -PI / 40, 0.33 * PI, -0.48 * PI, 0.33 * PI, -0.75 * PI, 0, 1, 0, 0, 0, 0, 0},
    {0, -0.1490, -PI / 25, 0.35 * PI, -0.7 * PI, 0.25 * PI, -0.60 * PI, 0, -1, 0, 0, 0, 0, 0}};
static __constant__ double cQjointBias[4] = {0.3 * PI, -0.7 * PI, 0.3 * PI, -0.7 * PI};
constexpr double kGRF = 8.252 * 9.81;  // ReferenceGen.cpp:27

static __device__ __forceinline__ double* traj_ptr(const SolveParams& sp, const DevBufs& d, int b,
                                            int slot, int kk) {
  return d.traj + (((size_t)b * sp.nslot + slot) * sp.NK + kk) * KS;
}

static __device__ __forceinline__ int ntc_of(int mode, bool wb) { return wb && (mode == 2 || mode == 4); }

// ---- reduced barrier (SinglePhase.cpp:298-317), k = 2 ---------------------------------
// The reference's pow() calls with integer exponents are evaluated exactly as products:
// pow(t, 2) = t*t (the correctly rounded square), pow(t, 1) = t, pow(t, 0) = 1 (also for
// NaN, as pow defines), pow(g, -2) = 1/(g*g) (within 1 ulp of the correctly rounded value).
static __device__ __forceinline__ void reduced_barrier(double g, double delta, double* B, double* Bz,
                                                double* Bzz) {
  if (g > delta) {
    *B = -log(g);
    *Bz = -1.0 / g;
    *Bzz = 1.0 / (g * g);
  } else {
    const double t = (g - 2 * delta) / ((2 - 1) * delta);
    *B = (double)(2 - 1) / 2 * (t * t - 1) - log(delta);
    *Bz = t / delta;
    *Bzz = 1.0;
  }
}

// Running cost value incl. the ReB barrier of WB phases (CostBase.cpp:4-16,
// SinglePhase.cpp:219-249 in CALC_DYNAMICS_ONLY), reference of knot kk built in registers.
static __device__ double wb_running_cost(const SolveParams& sp, int mode, double dt, double pos,
                                  const double* x, const double* u, const double* y, bool reb,
                                  double delta, double eps_tq, double eps_grf) {
  const int m = mode - 1;
  double rx[14] = {pos, sp.height, 0, cQjointBias[0], cQjointBias[1], cQjointBias[2],
                   cQjointBias[3], sp.vel, 0, 0, 0, 0, 0, 0};
  const double ry[4] = {0, kGRF, 0, kGRF};
  double l = 0, t = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i) { const double e = x[i] - rx[i]; l += e * cQwb[i] * e; }
#pragma unroll
  for (int i = 0; i < 4; ++i) { const double e = u[i]; t += e * cRwb[m][i] * e; }
  l += t;
  t = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) { const double e = y[i] - ry[i]; t += e * cSwb[m][i] * e; }
  l += t;
  l = l * dt;
  if (reb) {
    double B, Bz, Bzz;
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // torque limits 33 -/+ u
      const double g = (i < 4 ? -u[i] : u[i - 4]) + 33;
      reduced_barrier(g, delta, &B, &Bz, &Bzz);
      l += eps_tq * B * dt;
    }
    // joint limits carry eps_ReB = 0 (MHPCConstraints.cpp:64-84): contribution 0 * B * dt
    if (mode == 1 || mode == 3) {  // GRF: Fz >= 0, mu Fz -/+ Fx >= 0 with mu = 0.5
      const int o = mode == 1 ? 2 : 0;
      const double gs[3] = {y[o + 1], -y[o] + 0.5 * y[o + 1], y[o] + 0.5 * y[o + 1]};
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        reduced_barrier(gs[i], delta, &B, &Bz, &Bzz);
        l += eps_grf * B * dt;
      }
    }
  }
  return l;
}

static __device__ double fb_running_cost(const SolveParams& sp, int mode, double dt, double pos,
                                  const double* x, const double* u) {
  const int m = mode - 1;
  const double rx[6] = {pos, sp.height, 0, sp.vel, 0, 0};
  const double ru[4] = {0, kGRF, 0, kGRF};
  double l = 0, t = 0;
#pragma unroll
  for (int i = 0; i < 6; ++i) { const double e = x[i] - rx[i]; l += e * cQfb[i] * e; }
#pragma unroll
  for (int i = 0; i < 4; ++i) { const double e = u[i] - ru[i]; t += e * cRfb[m][i] * e; }
  l += t;
  l += 0.0;  // S = 0 for the floating base (y = 0)
  return l * dt;
}

// Derivatives of a WB running cost w.r.t. u and the stance force (CostBase.cpp:19-34 and
// the CALC_PARTIALS_ONLY branch of SinglePhase.cpp:219-249; joint limits carry eps_ReB = 0
// and contribute exact zeros).  out = lu[4], luu[4] (diagonal), ly[2], lyy[4] where ly/lyy
// are the entries of the stance foot's force slots (zero in flight).
static __device__ void wb_cost_uy_derivs(int mode, double dt, const double* u, const double* y,
                                         bool reb, double delta, double eps_tq, double eps_grf,
                                         double* out) {
  const int m = mode - 1;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    double lu = (2 * dt * cRwb[m][c]) * (u[c] - 0.0);
    double luu = 2 * dt * cRwb[m][c];
    if (reb) {
      double B, Bz, Bzz;
      // constraint c: g = -u_c + 33 (gu = -1); constraint 4 + c: g = u_c + 33 (gu = +1)
      reduced_barrier(-1.0 * u[c] + 33, delta, &B, &Bz, &Bzz);
      lu += eps_tq * Bz * -1.0 * dt;
      luu += eps_tq * (-1.0 * Bzz * -1.0) * dt;
      reduced_barrier(1.0 * u[c] + 33, delta, &B, &Bz, &Bzz);
      lu += eps_tq * Bz * 1.0 * dt;
      luu += eps_tq * (1.0 * Bzz * 1.0) * dt;
    }
    out[c] = lu;
    out[4 + c] = luu;
  }
  out[8] = out[9] = out[10] = out[11] = out[12] = out[13] = 0.0;
  if (mode == 1 || mode == 3) {
    const int o = mode == 1 ? 2 : 0;
    const double fx = mode == 1 ? y[2] : y[0], fz = mode == 1 ? y[3] : y[1];
    const double s0 = cSwb[m][o], s1 = cSwb[m][o + 1];
    double ly0 = (2 * dt * s0) * (fx - 0.0);
    double ly1 = (2 * dt * s1) * (fz - kGRF);
    double l00 = 2 * dt * s0, l01 = 0.0, l10 = 0.0, l11 = 2 * dt * s1;
    if (reb) {
      const double rows[3][2] = {{0, 1}, {-1, 0.5}, {1, 0.5}};  // coefficients on (Fx, Fz)
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        double B, Bz, Bzz;
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

static __device__ void wb_term_ref(const SolveParams& sp, int mode, double pos, double* rx) {
#pragma unroll
  for (int i = 0; i < 14; ++i) rx[i] = cXtermWB[mode - 1][i];
  rx[7] = sp.vel;
  rx[0] = pos;
}

static __device__ void fb_term_ref(const SolveParams& sp, double pos, double* rx) {
  rx[0] = pos; rx[1] = sp.height; rx[2] = 0; rx[3] = sp.vel; rx[4] = 0; rx[5] = 0;
}

// FootholdPlanner::get_foothold_location (FootholdPlan.h:26-50), velcmd 1.5 / ground
// -0.404 hard-coded by the reference (MHPCLocomotion.cpp:25).
static __device__ void plan_foothold(const double* x0, double stance_time, int mode, double* f) {
  f[0] = f[1] = f[2] = f[3] = 0;
  if (mode == 1) {
    f[2] = (cos(x0[2]) * (-0.19) + x0[0]) + 1.5 * stance_time / 2;
    f[3] = -0.404;
  } else if (mode == 3) {
    f[0] = (cos(x0[2]) * 0.19 + x0[0]) + 1.5 * stance_time / 2;
    f[1] = -0.404;
  }
}


}  // namespace mhpc
