// HIP kernels of the batched HSDDP solve for gfx950 (MI355X).
//
// One solve = a fixed host schedule of five kernels per DDP iteration (see
// mhpc_runtime.cpp), every kernel working on the whole batch and skipping problems whose
// per-problem state machine (ProbState) says they are done -- the divergent control flow
// of MultiPhaseDDP::solve (MultiPhaseDDP.cpp:154-289) lives in device memory, not on the
// host:
//   k_rollout  lane = (problem, line-search candidate).  forward_sweep(0) (FULL) or all
//              Armijo trials of forward_iteration (LS) at once, each lane a serial
//              multi-phase rollout with costs, barrier, AL and phase transitions; the
//              first accepted trial is selected in-wave (MultiPhaseDDP.cpp:130-151).
//   k_partials lane = (problem, knot, tangent direction): dual-number evaluation of the
//              whole-body model -> every column of A,B,C,D and of the impact Jacobian Px
//              in parallel (forward_sweep_partials_only, SinglePhase.cpp:147-180).
//   k_bws      one wavefront per problem: the backward Riccati sweep over all phases with
//              impact-aware steps and the regularisation-retry loop
//              (MultiPhaseDDP.cpp:100-127,196-241, SinglePhase.cpp:183-216,
//              MHPC_CompoundTypes.h:117-144).  Knot blocks (<= 14x14) are staged in LDS,
//              the 64 lanes split each product; no MFMA (blocks far below MFMA shapes).
//   k_al_end   AL / ReB parameter update and outer-loop exit (MultiPhaseDDP.cpp:273-284).
#include <hip/hip_runtime.h>

#include "mhpc_model.h"
#include "mhpc_solver.h"

namespace mhpc {

constexpr double PI = 3.141592653589793238;  // MHPC_CPPTypes.h:18

// ---- cost weights (MHPCCost.cpp:24-75) ------------------------------------------------
__constant__ double cQwb[14] = {0.01 * 0, 0.01 * 10, 0.01 * 5, 0.01 * 4, 0.01 * 4, 0.01 * 4,
                                0.01 * 4, 0.01 * 2, 0.01 * 1, 0.01 * .01, 0.01 * 6, 0.01 * 6,
                                0.01 * 6, 0.01 * 6};
__constant__ double cQfwb[4][14] = {
    {100 * 0., 100 * 20., 100 * 8., 100 * 3., 100 * 3., 100 * 3., 100 * 3., 100 * 3., 100 * 2.,
     100 * 0.01, 100 * 5., 100 * 5., 100 * 0.01, 100 * 0.01},
    {100 * 0., 100 * 20., 100 * 8., 100 * 3., 100 * 3., 100 * 3., 100 * 3., 100 * 3., 100 * 2.,
     100 * 0.01, 100 * 5., 100 * 5., 100 * 5., 100 * 5.},
    {100 * 0., 100 * 20., 100 * 8., 100 * 3., 100 * 3., 100 * 3., 100 * 3., 100 * 3., 100 * 2.,
     100 * 0.01, 100 * 0.01, 100 * 0.01, 100 * 5., 100 * 5.},
    {100 * 0., 100 * 20., 100 * 8., 100 * 3., 100 * 3., 100 * 3., 100 * 3., 100 * 3., 100 * 2.,
     100 * 0.01, 100 * 5., 100 * 5., 100 * 5., 100 * 5.}};
__constant__ double cRwb[4][4] = {{0.5 * 5, 0.5 * 5, 0.5 * 1, 0.5 * 1},
                                  {0.5 * 1, 0.5 * 1, 0.5 * 1, 0.5 * 1},
                                  {0.5 * 1, 0.5 * 1, 0.5 * 5, 0.5 * 5},
                                  {0.5 * 1, 0.5 * 1, 0.5 * 1, 0.5 * 1}};
// s[3] is uninitialised in the reference (MHPCCost.cpp:43 fills s[0..2]); zero here, as in
// the oracle.  It can only offset the value of WB mode-4 running costs (y = 0 in flight).
__constant__ double cSwb[4][4] = {{0, 0, 0.3, 0.3}, {0, 0, 0, 0}, {0.15, 0.15, 0, 0}, {0, 0, 0, 0}};
__constant__ double cQfb[6] = {0.01 * 0, 0.01 * 10, 0.01 * 5, 0.01 * 2, 0.01 * 1, 0.01 * 0.01};
__constant__ double cQffb[6] = {100 * 1., 100 * 20., 100 * 8., 100 * 3., 100 * 1., 100 * 0.01};
__constant__ double cRfb[4][4] = {{0, 0, 0.01, 0.01}, {0, 0, 0, 0}, {0.01, 0.01, 0, 0}, {0, 0, 0, 0}};
// terminal WB state references (ReferenceGen.cpp:45-52), velocity entry filled at run time
__constant__ double cXtermWB[4][14] = {
    {0, -0.1432, -PI / 25, 0.35 * PI, -0.65 * PI, 0.35 * PI, -0.6 * PI, 0, 1, 0, 0, 0, 0, 0},
    {0, -0.1418, PI / 35, 0.2 * PI, -0.58 * PI, 0.25 * PI, -0.7 * PI, 0, -1, 0, 0, 0, 0, 0},
    {0, -0.1325, -PI / 40, 0.33 * PI, -0.48 * PI, 0.33 * PI, -0.75 * PI, 0, 1, 0, 0, 0, 0, 0},
    {0, -0.1490, -PI / 25, 0.35 * PI, -0.7 * PI, 0.25 * PI, -0.60 * PI, 0, -1, 0, 0, 0, 0, 0}};
__constant__ double cQjointBias[4] = {0.3 * PI, -0.7 * PI, 0.3 * PI, -0.7 * PI};
constexpr double kGRF = 8.252 * 9.81;  // ReferenceGen.cpp:27

__device__ __forceinline__ double* traj_ptr(const SolveParams& sp, const DevBufs& d, int b,
                                            int slot, int kk) {
  return d.traj + (((size_t)b * sp.nslot + slot) * sp.NK + kk) * KS;
}

__device__ __forceinline__ int ntc_of(int mode, bool wb) { return wb && (mode == 2 || mode == 4); }

// ---- reduced barrier (SinglePhase.cpp:298-317), k = 2 ---------------------------------
__device__ __forceinline__ void reduced_barrier(double g, double delta, double* B, double* Bz,
                                                double* Bzz) {
  if (g > delta) {
    *B = -log(g);
    *Bz = -1.0 / g;
    *Bzz = pow(g, -2.0);
  } else {
    const double t = (g - 2 * delta) / ((2 - 1) * delta);
    *B = (double)(2 - 1) / 2 * (pow(t, 2.0) - 1) - log(delta);
    *Bz = pow(t, 1.0) / delta;
    *Bzz = pow(t, 0.0);
  }
}

// Running cost value incl. the ReB barrier of WB phases (CostBase.cpp:4-16,
// SinglePhase.cpp:219-249 in CALC_DYNAMICS_ONLY), reference of knot kk built in registers.
__device__ double wb_running_cost(const SolveParams& sp, int mode, double dt, double pos,
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

__device__ double fb_running_cost(const SolveParams& sp, int mode, double dt, double pos,
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

__device__ void wb_term_ref(const SolveParams& sp, int mode, double pos, double* rx) {
#pragma unroll
  for (int i = 0; i < 14; ++i) rx[i] = cXtermWB[mode - 1][i];
  rx[7] = sp.vel;
  rx[0] = pos;
}

__device__ void fb_term_ref(const SolveParams& sp, double pos, double* rx) {
  rx[0] = pos; rx[1] = sp.height; rx[2] = 0; rx[3] = sp.vel; rx[4] = 0; rx[5] = 0;
}

// FootholdPlanner::get_foothold_location (FootholdPlan.h:26-50), velcmd 1.5 / ground
// -0.404 hard-coded by the reference (MHPCLocomotion.cpp:25).
__device__ void plan_foothold(const double* x0, double stance_time, int mode, double* f) {
  f[0] = f[1] = f[2] = f[3] = 0;
  if (mode == 1) {
    f[2] = (cos(x0[2]) * (-0.19) + x0[0]) + 1.5 * stance_time / 2;
    f[3] = -0.404;
  } else if (mode == 3) {
    f[0] = (cos(x0[2]) * 0.19 + x0[0]) + 1.5 * stance_time / 2;
    f[1] = -0.404;
  }
}

// ============================================================================================
// k_rollout
// ============================================================================================
constexpr int RO_MAXP = MAXP;

__global__ __launch_bounds__(64) void k_rollout(SolveParams sp, DevBufs d, int full, int al_iter,
                                                int ddp_iter, int max_ddp) {
  const int nc = full ? 1 : sp.n_cand;
  const int ppw = 64 / nc;
  const int lane = threadIdx.x;
  const int lp = lane / nc, j = lane - lp * nc;
  const int b = blockIdx.x * ppw + lp;
  const bool in = lp < ppw && b < sp.B;

  __shared__ double sJ[64], sViol[64], sV[64][RO_MAXP], sH[64][RO_MAXP];
  __shared__ int sAcc[64];

  bool run = false;
  ProbState* st = nullptr;
  if (in) {
    st = &d.st[b];
    run = st->active && (full || st->ddp_active);
  }
  int nom = 0, slot = 0;
  double eps = 0;
  if (run) {
    if (full) {
      // top of the AL iteration (MultiPhaseDDP.cpp:172-190)
      const bool reb_off = (st->viol > 0.05) || al_iter == 1;
      st->reb_active = (sp.ReB_active && !reb_off) ? 1 : 0;
    }
    nom = st->nom_slot;
    slot = j < nom ? j : j + 1;
    eps = full ? 0.0 : sp.eps[j];
  }
  const bool reb = run && st->reb_active;
  double J = 0, viol2 = 0;
  if (run) {
    double x[14];
    const double* x0 = d.x0 + (size_t)b * 14;
    for (int i = 0; i < 14; ++i) x[i] = x0[i];
    for (int p = 0; p < sp.P; ++p) {
      const int mode = sp.mode[p], N = sp.N[p], ko = sp.ko[p];
      const double dt = sp.dt[p];
      double V = 0, h = 0;
      const double* refpos = d.refpos + (size_t)b * sp.NK + ko;
      if (p < sp.n_wb) {
        const double delta = st->delta[p], etq = st->eps_tq[p], egr = st->eps_grf[p];
        for (int k = 0; k < N - 1; ++k) {
          const double* nk = traj_ptr(sp, d, b, nom, ko + k);
          const double* Kk = d.K + ((size_t)b * sp.NK + ko + k) * 56;
          const double* duk = d.du + ((size_t)b * sp.NK + ko + k) * 4;
          double u[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            double fb = 0;
#pragma unroll
            for (int c = 0; c < 14; ++c) fb += Kk[i * 14 + c] * (x[c] - nk[c]);
            u[i] = (nk[14 + i] + eps * duk[i]) + fb;
          }
          double xd[14], y[4];
          wb_dynamics<double>(x, u, mode, xd, y);
          V += wb_running_cost(sp, mode, dt, refpos[k], x, u, y, reb, delta, etq, egr);
          double* ok = traj_ptr(sp, d, b, slot, ko + k);
#pragma unroll
          for (int i = 0; i < 14; ++i) ok[i] = x[i];
#pragma unroll
          for (int i = 0; i < 4; ++i) { ok[14 + i] = u[i]; ok[18 + i] = y[i]; }
#pragma unroll
          for (int i = 0; i < 14; ++i) x[i] = x[i] + xd[i] * dt;
        }
        double* oe = traj_ptr(sp, d, b, slot, ko + N - 1);
        for (int i = 0; i < 14; ++i) oe[i] = x[i];
        // terminal cost, constraint and AL (CostBase.cpp:37-47, SinglePhase.cpp:257-275)
        double rx[14];
        wb_term_ref(sp, mode, refpos[N - 1], rx);
        double Phi = 0;
        for (int i = 0; i < 14; ++i) { const double e = x[i] - rx[i]; Phi += e * cQfwb[mode - 1][i] * e; }
        Phi = Phi * 0.5;
        if (ntc_of(mode, true)) {
          h = wb_touchdown_value(x, mode == 2 ? kFront : kBack);
          if (sp.AL_active) {
            const double s = st->sigma[p], lam = st->lambda[p];
            Phi += 50 * (pow(s * h / 2, 2.0) + lam * h);
          }
        }
        V += Phi;
        // phase transition (MultiPhaseDDP.cpp:351-379)
        if (p + 1 < sp.P) {
          if (mode == 2 || mode == 4) {
            double xp[14], lam[2];
            wb_impact<double>(x, mode == 2 ? kFront : kBack, xp, lam);
            for (int i = 0; i < 14; ++i) x[i] = xp[i];
          }
          if (p + 1 >= sp.n_wb) {
            const double t0 = x[0], t1 = x[1], t2 = x[2], t7 = x[7], t8 = x[8], t9 = x[9];
            x[0] = t0; x[1] = t1; x[2] = t2; x[3] = t7; x[4] = t8; x[5] = t9;
          }
        }
      } else {
        double f[4], s[2];
        plan_foothold(x, dt * N, mode, f);
        srb_contact(mode, s);
        for (int k = 0; k < N - 1; ++k) {
          const double* nk = traj_ptr(sp, d, b, nom, ko + k);
          const double* Kk = d.K + ((size_t)b * sp.NK + ko + k) * 56;
          const double* duk = d.du + ((size_t)b * sp.NK + ko + k) * 4;
          double u[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            double fb = 0;
#pragma unroll
            for (int c = 0; c < 6; ++c) fb += Kk[i * 6 + c] * (x[c] - nk[c]);
            u[i] = (nk[6 + i] + eps * duk[i]) + fb;
          }
          double xd[6];
          srb_dynamics(x, u, f, s, xd);
          V += fb_running_cost(sp, mode, dt, refpos[k], x, u);
          double* ok = traj_ptr(sp, d, b, slot, ko + k);
#pragma unroll
          for (int i = 0; i < 6; ++i) ok[i] = x[i];
#pragma unroll
          for (int i = 0; i < 4; ++i) { ok[6 + i] = u[i]; ok[10 + i] = 0.0; }
#pragma unroll
          for (int i = 0; i < 6; ++i) x[i] = x[i] + xd[i] * dt;
        }
        double* oe = traj_ptr(sp, d, b, slot, ko + N - 1);
        for (int i = 0; i < 6; ++i) oe[i] = x[i];
        double rx[6];
        fb_term_ref(sp, refpos[N - 1], rx);
        double Phi = 0;
        for (int i = 0; i < 6; ++i) { const double e = x[i] - rx[i]; Phi += e * cQffb[i] * e; }
        V += Phi * 0.5;
      }
      J += V;
      viol2 += h * h;
      sV[lane][p] = V;
      sH[lane][p] = h;
    }
    sJ[lane] = J;
    sViol[lane] = sqrt(viol2);
    const double cost_prev = st->J;
    const double rhs = cost_prev + sp.gamma * eps * (1 - eps / 2) * st->dV_exp;
    sAcc[lane] = full ? 1 : (sJ[lane] <= rhs ? 1 : 0);
  }
  __syncthreads();
  if (run && j == 0) {
    int sel = nc - 1, nls = nc + 1;
    for (int c = 0; c < nc; ++c)
      if (sAcc[lane + c]) { sel = c; nls = c + 1; break; }
    const int sl = lane + sel;
    const double cost_prev = st->J;
    st->J = sJ[sl];
    st->viol = sViol[sl];
    for (int p = 0; p < sp.P; ++p) { st->V[p] = sV[sl][p]; st->h[p] = sH[sl][p]; }
    st->nom_slot = sel < nom ? sel : sel + 1;
    if (full) {
      st->al_iter = al_iter;
      st->reg = 0;
      st->ddp_active = 1;
      st->al_partials = 1;
      st->cnt[C_FWD]++;
      st->cnt[C_PAR_RUN]++;
    } else {
      const bool conv = cost_prev - st->J < sp.DDP_thresh;
      if (st->ntrace < TRACE)
        st->trace[st->ntrace++] = (al_iter << 24) | (st->reb_active << 23) | ((conv ? 1 : 0) << 22) |
                                  ((nls & 0xff) << 8) | (st->bws_iter & 0xff);
      st->cnt[C_LS] += nls < nc ? nls : nc;
      st->cnt[C_LS_RUN] += nc;
      st->cnt[C_LS_LAUNCH]++;
      if (conv) {
        st->ddp_active = 0;
      } else {
        st->cnt[C_PAR]++;
        st->al_partials = 0;
        if (ddp_iter < max_ddp) st->cnt[C_PAR_RUN]++;
        else st->ddp_active = 0;
      }
    }
  }
}

// ============================================================================================
// k_partials: one lane per (problem, knot, tangent direction)
// ============================================================================================
__global__ __launch_bounds__(256) void k_partials(SolveParams sp, DevBufs d) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int b = (int)(t / sp.par_items);
  if (b >= sp.B) return;
  const int it = (int)(t - (long)b * sp.par_items);
  const ProbState* st = &d.st[b];
  if (!(st->active && st->ddp_active)) return;
  int p = 0;
  while (it >= sp.par_item_off[p + 1]) ++p;
  const int loc = it - sp.par_item_off[p];
  const int N = sp.N[p], ko = sp.ko[p], mode = sp.mode[p];
  const int nom = st->nom_slot;
  if (loc < (N - 1) * 18) {
    const int k = loc / 18, dir = loc - k * 18;
    const double* nk = traj_ptr(sp, d, b, nom, ko + k);
    Dual x[14], u[4], f[14], y[4];
#pragma unroll
    for (int i = 0; i < 14; ++i) x[i] = Dual(nk[i], i == dir ? 1.0 : 0.0);
#pragma unroll
    for (int i = 0; i < 4; ++i) u[i] = Dual(nk[14 + i], 14 + i == dir ? 1.0 : 0.0);
    wb_dynamics<Dual>(x, u, mode, f, y);
    double* out = d.par + ((size_t)b * sp.NK + ko + k) * PS + dir * 9;
#pragma unroll
    for (int i = 0; i < 7; ++i) out[i] = f[7 + i].d;
    const int o = mode == 1 ? 2 : 0;
    out[7] = y[o].d;
    out[8] = y[o + 1].d;
  } else {
    const int dir = loc - (N - 1) * 18;
    const double* nk = traj_ptr(sp, d, b, nom, ko + N - 1);
    Dual x[14], xp[14], lam[2];
#pragma unroll
    for (int i = 0; i < 14; ++i) x[i] = Dual(nk[i], i == dir ? 1.0 : 0.0);
    wb_impact<Dual>(x, mode == 2 ? kFront : kBack, xp, lam);
    double* out = d.px + ((size_t)b * MAXP + p) * 196 + dir * 14;
#pragma unroll
    for (int i = 0; i < 14; ++i) out[i] = xp[i].d;
  }
}

// ============================================================================================
// k_bws: one wavefront per problem
// ============================================================================================
struct BwsLds {
  double H[196], G[14];            // value function of knot k+1, then of knot k
  double A[196], Bm[56], C[56], D[16];
  double lx[14], lxx[14], luu[16], lyy[16];
  double T[196], BtH[56], Ctl[56], Dtl[16];
  double Qx[14], Qu[4], Qxx[196], Quu[16], Qux[56];
  double tq[56];                   // Qux' * Quu_inv   (n x 4)
  double xb[14], ub[4], yb[4];     // nominal knot
  double P[PS];                    // partials record of the knot
  double Px[196];
  double G2[14], H2[196];          // impact-aware step scratch
};

// Eigen-style 4x4 inverse by cofactors (same formulas as the oracle).
__device__ void inverse4(const double* m, double* inv) {
  double a[16];
  a[0] = m[5] * m[10] * m[15] - m[5] * m[11] * m[14] - m[9] * m[6] * m[15] + m[9] * m[7] * m[14] +
         m[13] * m[6] * m[11] - m[13] * m[7] * m[10];
  a[4] = -m[4] * m[10] * m[15] + m[4] * m[11] * m[14] + m[8] * m[6] * m[15] - m[8] * m[7] * m[14] -
         m[12] * m[6] * m[11] + m[12] * m[7] * m[10];
  a[8] = m[4] * m[9] * m[15] - m[4] * m[11] * m[13] - m[8] * m[5] * m[15] + m[8] * m[7] * m[13] +
         m[12] * m[5] * m[11] - m[12] * m[7] * m[9];
  a[12] = -m[4] * m[9] * m[14] + m[4] * m[10] * m[13] + m[8] * m[5] * m[14] - m[8] * m[6] * m[13] -
          m[12] * m[5] * m[10] + m[12] * m[6] * m[9];
  a[1] = -m[1] * m[10] * m[15] + m[1] * m[11] * m[14] + m[9] * m[2] * m[15] - m[9] * m[3] * m[14] -
         m[13] * m[2] * m[11] + m[13] * m[3] * m[10];
  a[5] = m[0] * m[10] * m[15] - m[0] * m[11] * m[14] - m[8] * m[2] * m[15] + m[8] * m[3] * m[14] +
         m[12] * m[2] * m[11] - m[12] * m[3] * m[10];
  a[9] = -m[0] * m[9] * m[15] + m[0] * m[11] * m[13] + m[8] * m[1] * m[15] - m[8] * m[3] * m[13] -
         m[12] * m[1] * m[11] + m[12] * m[3] * m[9];
  a[13] = m[0] * m[9] * m[14] - m[0] * m[10] * m[13] - m[8] * m[1] * m[14] + m[8] * m[2] * m[13] +
          m[12] * m[1] * m[10] - m[12] * m[2] * m[9];
  a[2] = m[1] * m[6] * m[15] - m[1] * m[7] * m[14] - m[5] * m[2] * m[15] + m[5] * m[3] * m[14] +
         m[13] * m[2] * m[7] - m[13] * m[3] * m[6];
  a[6] = -m[0] * m[6] * m[15] + m[0] * m[7] * m[14] + m[4] * m[2] * m[15] - m[4] * m[3] * m[14] -
         m[12] * m[2] * m[7] + m[12] * m[3] * m[6];
  a[10] = m[0] * m[5] * m[15] - m[0] * m[7] * m[13] - m[4] * m[1] * m[15] + m[4] * m[3] * m[13] +
          m[12] * m[1] * m[7] - m[12] * m[3] * m[5];
  a[14] = -m[0] * m[5] * m[14] + m[0] * m[6] * m[13] + m[4] * m[1] * m[14] - m[4] * m[2] * m[13] -
          m[12] * m[1] * m[6] + m[12] * m[2] * m[5];
  a[3] = -m[1] * m[6] * m[11] + m[1] * m[7] * m[10] + m[5] * m[2] * m[11] - m[5] * m[3] * m[10] -
         m[9] * m[2] * m[7] + m[9] * m[3] * m[6];
  a[7] = m[0] * m[6] * m[11] - m[0] * m[7] * m[10] - m[4] * m[2] * m[11] + m[4] * m[3] * m[10] +
         m[8] * m[2] * m[7] - m[8] * m[3] * m[6];
  a[11] = -m[0] * m[5] * m[11] + m[0] * m[7] * m[9] + m[4] * m[1] * m[11] - m[4] * m[3] * m[9] -
          m[8] * m[1] * m[7] + m[8] * m[3] * m[5];
  a[15] = m[0] * m[5] * m[10] - m[0] * m[6] * m[9] - m[4] * m[1] * m[10] + m[4] * m[2] * m[9] +
          m[8] * m[1] * m[6] - m[8] * m[2] * m[5];
  const double det = m[0] * a[0] + m[1] * a[4] + m[2] * a[8] + m[3] * a[12];
#pragma unroll
  for (int i = 0; i < 16; ++i) inv[i] = a[i] / det;
}

// Eigen LDLT(...).isPositive() on the lower triangle of a 4x4 (see oracle).
__device__ bool ldlt_is_positive4(const double* Ain) {
  double A[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) A[i] = Ain[i];
  int sign = 0;  // 0 ZeroSign, 1 PositiveSemiDef, 2 NegativeSemiDef, 3 Indefinite
  double temp[4];
  for (int k = 0; k < 4; ++k) {
    int big = k;
    double bigv = fabs(A[k * 4 + k]);
    for (int i = k + 1; i < 4; ++i)
      if (fabs(A[i * 4 + i]) > bigv) { bigv = fabs(A[i * 4 + i]); big = i; }
    if (big != k) {
      for (int jj = 0; jj < k; ++jj) { const double t = A[k * 4 + jj]; A[k * 4 + jj] = A[big * 4 + jj]; A[big * 4 + jj] = t; }
      for (int i = big + 1; i < 4; ++i) { const double t = A[i * 4 + k]; A[i * 4 + k] = A[i * 4 + big]; A[i * 4 + big] = t; }
      { const double t = A[k * 4 + k]; A[k * 4 + k] = A[big * 4 + big]; A[big * 4 + big] = t; }
      for (int i = k + 1; i < big; ++i) { const double t = A[i * 4 + k]; A[i * 4 + k] = A[big * 4 + i]; A[big * 4 + i] = t; }
    }
    if (k > 0) {
      for (int jj = 0; jj < k; ++jj) temp[jj] = A[jj * 4 + jj] * A[k * 4 + jj];
      double s = 0;
      for (int jj = 0; jj < k; ++jj) s += A[k * 4 + jj] * temp[jj];
      A[k * 4 + k] -= s;
      for (int i = k + 1; i < 4; ++i) {
        double t = 0;
        for (int jj = 0; jj < k; ++jj) t += A[i * 4 + jj] * temp[jj];
        A[i * 4 + k] -= t;
      }
    }
    const double akk = A[k * 4 + k];
    const bool valid = fabs(akk) > 0.0;
    if (k == 0 && !valid) { sign = 0; break; }
    if (k < 3 && valid)
      for (int i = k + 1; i < 4; ++i) A[i * 4 + k] /= akk;
    if (sign == 1) { if (akk < 0.0) sign = 3; }
    else if (sign == 2) { if (akk > 0.0) sign = 3; }
    else if (sign == 0) { if (akk > 0.0) sign = 1; else if (akk < 0.0) sign = 2; }
  }
  return sign == 1 || sign == 0;
}

// Per-knot cost derivatives, identical for every lane (registers): lu, ly, luu(diag), lyy.
// lx / lxx per state index are produced by the caller's lanes.  CostBase.cpp:19-34 +
// SinglePhase.cpp:219-249 (CALC_PARTIALS_ONLY / DYN_AND_PAR branch).
__device__ void wb_cost_uy(int mode, double dt, const double* u, const double* y, bool reb,
                           double delta, double eps_tq, double eps_grf, double* lu, double* ly,
                           double* luu, double* lyy) {
  const int m = mode - 1;
  const double c = 2 * dt;
  const double ry[4] = {0, kGRF, 0, kGRF};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    lu[i] = (c * cRwb[m][i]) * (u[i] - 0.0);
    ly[i] = (c * cSwb[m][i]) * (y[i] - ry[i]);
    luu[i] = c * cRwb[m][i];
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) lyy[i] = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) lyy[i * 5] = c * cSwb[m][i];
  if (!reb) return;
  double B, Bz, Bzz;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int a = i & 3;
    const double gu = i < 4 ? -1.0 : 1.0;
    const double g = gu * u[a] + 33;
    reduced_barrier(g, delta, &B, &Bz, &Bzz);
    lu[a] += eps_tq * Bz * gu * dt;
    luu[a] += eps_tq * (gu * Bzz * gu) * dt;
  }
  if (mode == 1 || mode == 3) {
    const int o = mode == 1 ? 2 : 0;
    const double rows[3][2] = {{0, 1}, {-1, 0.5}, {1, 0.5}};  // coefficients on (Fx, Fz)
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double g = rows[i][0] * y[o] + rows[i][1] * y[o + 1] + 0;
      reduced_barrier(g, delta, &B, &Bz, &Bzz);
#pragma unroll
      for (int a = 0; a < 2; ++a) ly[o + a] += eps_grf * Bz * rows[i][a] * dt;
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int c2 = 0; c2 < 2; ++c2)
          lyy[(o + a) * 4 + o + c2] += eps_grf * (rows[i][a] * Bzz * rows[i][c2]) * dt;
    }
  }
}

// One backward Riccati knot with NX states (compute_Qfunction + regularisation + PSD test
// + valuefunction_update).  sh.{A,Bm,C,D,lxx,luu,lyy} and lane-private lx_l/lu/ly hold the
// knot's derivatives (lx in sh.lx); sh.H/G hold the value function of knot k+1 and
// receive that of k.
template <int NX, bool HAS_Y>
__device__ bool riccati_knot(BwsLds& sh, int lane, const double* lu,
                             const double* ly, double reg, double eps9, double* Kout,
                             double* duout, double* Gout, double* dV) {
  constexpr int N2 = NX * NX, N4 = 4 * NX;
  // R2: T = A'H, BtH = B'H, Ctl = C'lyy, Dtl = D'lyy, Qx, Qu
  for (int e = lane; e < N2 + N4 + N4 + 16 + NX + 4; e += 64) {
    if (e < N2) {
      const int i = e / NX, jj = e - i * NX;
      double s = 0;
#pragma unroll
      for (int m = 0; m < NX; ++m) s += sh.A[m * NX + i] * sh.H[m * NX + jj];
      sh.T[e] = s;
    } else if (e < N2 + N4) {
      const int q = e - N2, c = q / NX, jj = q - c * NX;
      double s = 0;
#pragma unroll
      for (int m = 0; m < NX; ++m) s += sh.Bm[m * 4 + c] * sh.H[m * NX + jj];
      sh.BtH[q] = s;
    } else if (e < N2 + 2 * N4) {
      const int q = e - N2 - N4, i = q / 4, c = q - i * 4;
      double s = 0;
      if (HAS_Y) {
#pragma unroll
        for (int r = 0; r < 4; ++r) s += sh.C[r * NX + i] * sh.lyy[r * 4 + c];
      }
      sh.Ctl[q] = s;
    } else if (e < N2 + 2 * N4 + 16) {
      const int q = e - N2 - 2 * N4, c = q / 4, c2 = q - c * 4;
      double s = 0;
      if (HAS_Y) {
#pragma unroll
        for (int r = 0; r < 4; ++r) s += sh.D[r * 4 + c] * sh.lyy[r * 4 + c2];
      }
      sh.Dtl[q] = s;
    } else if (e < N2 + 2 * N4 + 16 + NX) {
      const int i = e - (N2 + 2 * N4 + 16);
      double s = 0, s2 = 0;
#pragma unroll
      for (int m = 0; m < NX; ++m) s += sh.A[m * NX + i] * sh.G[m];
      if (HAS_Y) {
#pragma unroll
        for (int r = 0; r < 4; ++r) s2 += sh.C[r * NX + i] * ly[r];
      }
      sh.Qx[i] = (sh.lx[i] + s) + s2;
    } else {
      const int c = e - (N2 + 2 * N4 + 16 + NX);
      double s = 0, s2 = 0;
#pragma unroll
      for (int m = 0; m < NX; ++m) s += sh.Bm[m * 4 + c] * sh.G[m];
      if (HAS_Y) {
#pragma unroll
        for (int r = 0; r < 4; ++r) s2 += sh.D[r * 4 + c] * ly[r];
      }
      sh.Qu[c] = (lu[c] + s) + s2;
    }
  }
  __syncthreads();
  // R3: Qxx = (lxx + Ctl C) + T A ; Quu = (luu + Dtl D) + BtH B ; Qux = Dtl C + BtH A
  for (int e = lane; e < N2 + 16 + N4; e += 64) {
    if (e < N2) {
      const int i = e / NX, jj = e - i * NX;
      double s = 0, s2 = 0;
      if (HAS_Y) {
#pragma unroll
        for (int c = 0; c < 4; ++c) s += sh.Ctl[i * 4 + c] * sh.C[c * NX + jj];
      }
#pragma unroll
      for (int m = 0; m < NX; ++m) s2 += sh.T[i * NX + m] * sh.A[m * NX + jj];
      double v = ((i == jj ? sh.lxx[i] : 0.0) + s) + s2;
      if (i == jj) v += 1.0 * reg;
      sh.Qxx[e] = v;
    } else if (e < N2 + 16) {
      const int q = e - N2, c = q / 4, c2 = q - c * 4;
      double s = 0, s2 = 0;
      if (HAS_Y) {
#pragma unroll
        for (int r = 0; r < 4; ++r) s += sh.Dtl[c * 4 + r] * sh.D[r * 4 + c2];
      }
#pragma unroll
      for (int m = 0; m < NX; ++m) s2 += sh.BtH[c * NX + m] * sh.Bm[m * 4 + c2];
      double v = (sh.luu[q] + s) + s2;
      if (c == c2) v += 1.0 * reg;
      sh.Quu[q] = v;
    } else {
      const int q = e - N2 - 16, c = q / NX, jj = q - c * NX;
      double s = 0, s2 = 0;
      if (HAS_Y) {
#pragma unroll
        for (int r = 0; r < 4; ++r) s += sh.Dtl[c * 4 + r] * sh.C[r * NX + jj];
      }
#pragma unroll
      for (int m = 0; m < NX; ++m) s2 += sh.BtH[c * NX + m] * sh.A[m * NX + jj];
      sh.Qux[q] = (0.0 + s) + s2;
    }
  }
  __syncthreads();
  // R4 (all lanes, registers): PSD test of Quu - 1e-9 I, inverse, du, dV
  double Quu[16], Qr[16], inv[16], Qi[16], Qu[4];
#pragma unroll
  for (int i = 0; i < 16; ++i) { Quu[i] = sh.Quu[i]; Qr[i] = Quu[i] - ((i % 5 == 0) ? 1.0 * eps9 : 0.0); }
  if (!ldlt_is_positive4(Qr)) return false;
  inverse4(Quu, inv);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int c = 0; c < 4; ++c) Qi[i * 4 + c] = (inv[i * 4 + c] + inv[c * 4 + i]) / 2;
#pragma unroll
  for (int i = 0; i < 4; ++i) Qu[i] = sh.Qu[i];
  {
    double r[4], s = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      double t = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) t += Qu[k] * inv[k * 4 + c];
      r[c] = t;
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) s += r[c] * Qu[c];
    *dV += -s;
  }
  if (lane < 4) {
    double s = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) s += -Qi[lane * 4 + c] * Qu[c];
    duout[lane] = s;
  }
  // K = -Quu_inv Qux (4 x NX) and tq = Qux' Quu_inv (NX x 4)
  for (int e = lane; e < 2 * N4; e += 64) {
    if (e < N4) {
      const int c = e / NX, jj = e - c * NX;
      double s = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) s += -Qi[c * 4 + k] * sh.Qux[k * NX + jj];
      Kout[e] = s;
    } else {
      const int q = e - N4, i = q / 4, c = q - i * 4;
      double s = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) s += sh.Qux[k * NX + i] * Qi[k * 4 + c];
      sh.tq[q] = s;
    }
  }
  __syncthreads();
  // R5: H = sym(Qxx) - tq Qux ; G = Qx - tq Qu
  for (int e = lane; e < N2 + NX; e += 64) {
    if (e < N2) {
      const int i = e / NX, jj = e - i * NX;
      double s = 0;
#pragma unroll
      for (int c = 0; c < 4; ++c) s += sh.tq[i * 4 + c] * sh.Qux[c * NX + jj];
      sh.H[e] = (sh.Qxx[e] + sh.Qxx[jj * NX + i]) / 2 - s;
    } else {
      const int i = e - N2;
      double s = 0;
#pragma unroll
      for (int c = 0; c < 4; ++c) s += sh.tq[i * 4 + c] * Qu[c];
      const double g = sh.Qx[i] - s;
      sh.G[i] = g;
      Gout[i] = g;
    }
  }
  __syncthreads();
  return true;
}

// Terminal value function of phase p at its last knot (SinglePhase.cpp:189-191):
// G = Phix + Gnext, H = Phixx + Hnext with Gnext/Hnext in sh.G/sh.H on entry.
template <int NX>
__device__ void terminal_value(const SolveParams& sp, const ProbState* st, BwsLds& sh, int lane,
                               int p, bool wb, double pos, const double* xe, double* Gout) {
  const int mode = sp.mode[p];
  double rx[14];
  if (wb) wb_term_ref(sp, mode, pos, rx);
  else fb_term_ref(sp, pos, rx);
  const bool al = wb && ntc_of(mode, true) && sp.AL_active && st->al_partials;
  double h = 0, hx[14], Hs[3][3];
  int id[3] = {0, 0, 0};
  if (al) wb_touchdown_compact(xe, mode == 2 ? kFront : kBack, &h, hx, id, Hs);
  const double s = st->sigma[p], lam = st->lambda[p];
  for (int e = lane; e < NX * NX + NX; e += 64) {
    if (e < NX * NX) {
      const int i = e / NX, jj = e - i * NX;
      double v = i == jj ? (wb ? cQfwb[mode - 1][i] : cQffb[i]) : 0.0;
      if (al) {
        double hij = 0;
        for (int a = 0; a < 3; ++a)
          for (int c = 0; c < 3; ++c)
            if (id[a] == i && id[c] == jj) hij = Hs[a][c];
        v += 50 * (s * s / 2 * (hx[i] * hx[jj] + h * hij) + lam * hij);
      }
      sh.H[e] = v + sh.H[e];
    } else {
      const int i = e - NX * NX;
      double v = (wb ? cQfwb[mode - 1][i] : cQffb[i]) * (xe[i] - rx[i]);
      if (al) v += 50 * (s * s / 2 * hx[i] * h + lam * hx[i]);
      const double g = v + sh.G[i];
      sh.G[i] = g;
      Gout[i] = g;
    }
  }
  __syncthreads();
}

__device__ bool bws_sweep(const SolveParams& sp, const DevBufs& d, int b, ProbState* st,
                          BwsLds& sh, double reg, int64_t* knots, int64_t* knots_wb,
                          int64_t* px_reads) {
  const int lane = threadIdx.x;
  const int nom = st->nom_slot;
  double dVnext = 0;
  // Gnext = 0, Hnext = 0 for the last phase
  for (int e = lane; e < 196; e += 64) sh.H[e] = 0;
  if (lane < 14) sh.G[lane] = 0;
  __syncthreads();
  for (int p = sp.P - 1; p >= 0; --p) {
    const bool wb = p < sp.n_wb;
    const int N = sp.N[p], ko = sp.ko[p], mode = sp.mode[p];
    const double dt = sp.dt[p];
    if (p + 1 < sp.P) {
      // impact_aware_step (MultiPhaseDDP.cpp:300-341); sh.G/H hold CTG[0] of phase p+1
      dVnext = st->dV[p + 1];
      if (wb) {
        const bool nwb = p + 1 < sp.n_wb;
        const bool imp = mode == 2 || mode == 4;
        if (imp) {
          const double* pxc = d.px + ((size_t)b * MAXP + p) * 196;  // column-major
          for (int e = lane; e < 196; e += 64) sh.Px[(e % 14) * 14 + e / 14] = pxc[e];
          ++*px_reads;
        } else {
          for (int e = lane; e < 196; e += 64) sh.Px[e] = (e / 14 == e % 14) ? 1.0 : 0.0;
        }
        // lift G', H' of the next phase to the 14-dim full-model space: E' G', E' H' E
        // (E = _stateProj for an SRB next phase, identity otherwise)
        __syncthreads();
        for (int e = lane; e < 196 + 14; e += 64) {
          if (e < 196) {
            const int i = e / 14, jj = e % 14;
            double v = 0;
            if (nwb) v = sh.H[e];
            else {
              int pi = -1, pj = -1;
              for (int q = 0; q < 6; ++q) {
                const int r = q < 3 ? q : q + 4;
                if (r == i) pi = q;
                if (r == jj) pj = q;
              }
              v = (pi >= 0 && pj >= 0) ? sh.H[pi * 6 + pj] : 0.0;
            }
            sh.H2[e] = v;
          } else {
            const int i = e - 196;
            double v = 0;
            if (nwb) v = sh.G[i];
            else {
              const int q = i < 3 ? i : (i >= 7 && i < 10 ? i - 4 : -1);
              v = q >= 0 ? sh.G[q] : 0.0;
            }
            sh.G2[i] = v;
          }
        }
        __syncthreads();
        if (imp) {
          // G = Px' G2 ; T = Px' H2 ; H = T Px
          for (int e = lane; e < 196 + 14; e += 64) {
            if (e < 196) {
              const int i = e / 14, jj = e % 14;
              double s = 0;
              for (int m = 0; m < 14; ++m) s += sh.Px[m * 14 + i] * sh.H2[m * 14 + jj];
              sh.T[e] = s;
            } else {
              const int i = e - 196;
              double s = 0;
              for (int m = 0; m < 14; ++m) s += sh.Px[m * 14 + i] * sh.G2[m];
              sh.G[i] = s;
            }
          }
          __syncthreads();
          for (int e = lane; e < 196; e += 64) {
            const int i = e / 14, jj = e % 14;
            double s = 0;
            for (int m = 0; m < 14; ++m) s += sh.T[i * 14 + m] * sh.Px[m * 14 + jj];
            sh.H[e] = s;
          }
        } else {
          for (int e = lane; e < 196; e += 64) sh.H[e] = sh.H2[e];
          if (lane < 14) sh.G[lane] = sh.G2[lane];
        }
        __syncthreads();
      }
      // SRB current phase: G = G', H = H' (already in place)
    }
    double dV = dVnext;
    const double* pos = d.refpos + (size_t)b * sp.NK + ko;
    double* Gp = d.G + ((size_t)b * sp.NK + ko) * 14;
    const double* xe = traj_ptr(sp, d, b, nom, ko + N - 1);
    if (wb) terminal_value<14>(sp, st, sh, lane, p, true, pos[N - 1], xe, Gp + (size_t)(N - 1) * 14);
    else terminal_value<6>(sp, st, sh, lane, p, false, pos[N - 1], xe, Gp + (size_t)(N - 1) * 14);
    double foot[4] = {0, 0, 0, 0}, cs[2] = {0, 0};
    if (!wb) {
      plan_foothold(traj_ptr(sp, d, b, nom, ko), dt * N, mode, foot);
      srb_contact(mode, cs);
    }
    const bool reb = st->reb_active;
    const double delta = st->delta[p], etq = st->eps_tq[p], egr = st->eps_grf[p];
    for (int k = N - 2; k >= 0; --k) {
      const int kk = ko + k;
      const double* nk = traj_ptr(sp, d, b, nom, kk);
      double* Kout = d.K + ((size_t)b * sp.NK + kk) * 56;
      double* duout = d.du + ((size_t)b * sp.NK + kk) * 4;
      double* Gout = d.G + ((size_t)b * sp.NK + kk) * 14;
      bool ok;
      if (wb) {
        const double* prec = d.par + ((size_t)b * sp.NK + kk) * PS;
        for (int e = lane; e < PS; e += 64) sh.P[e] = prec[e];
        if (lane < 22) {
          const double v = nk[lane];
          if (lane < 14) sh.xb[lane] = v;
          else if (lane < 18) sh.ub[lane - 14] = v;
          else sh.yb[lane - 18] = v;
        }
        __syncthreads();
        // A = I + dt Ac, B = dt Bc, C, D (PlanarQuadruped.cpp:51-52)
        const int o = mode == 1 ? 2 : 0;
        const bool stance = mode == 1 || mode == 3;
        for (int e = lane; e < 196 + 56 + 56 + 16; e += 64) {
          if (e < 196) {
            const int i = e / 14, jj = e % 14;
            const double ac = i < 7 ? (jj == i + 7 ? 1.0 : 0.0) : sh.P[jj * 9 + (i - 7)];
            sh.A[e] = (i == jj ? 1.0 : 0.0) + ac * dt;
          } else if (e < 252) {
            const int q = e - 196, i = q / 4, c = q % 4;
            sh.Bm[q] = (i < 7 ? 0.0 : sh.P[(14 + c) * 9 + (i - 7)]) * dt;
          } else if (e < 308) {
            const int q = e - 252, r = q / 14, jj = q % 14;
            sh.C[q] = (stance && (r == o || r == o + 1)) ? sh.P[jj * 9 + 7 + (r - o)] : 0.0;
          } else {
            const int q = e - 308, r = q / 4, c = q % 4;
            sh.D[q] = (stance && (r == o || r == o + 1)) ? sh.P[(14 + c) * 9 + 7 + (r - o)] : 0.0;
          }
        }
        double lu[4], ly[4], luu[4], lyy[16];
        wb_cost_uy(mode, dt, sh.ub, sh.yb, reb, delta, etq, egr, lu, ly, luu, lyy);
        // lx, lxx (CostBase.cpp:28-31) for state index = lane
        double lx_l = 0;
        {
          const int i = lane < 14 ? lane : 0;
          const double rxi = i == 0 ? pos[k] : i == 1 ? sp.height : i == 2 ? 0.0
                             : i < 7 ? cQjointBias[i - 3] : i == 7 ? sp.vel : 0.0;
          lx_l = (2 * dt * cQwb[i]) * (sh.xb[i] - rxi);
          if (lane < 14) sh.lxx[lane] = 2 * dt * cQwb[lane];
        }
        if (lane < 16) {
          sh.luu[lane] = (lane % 5 == 0) ? luu[lane / 5] : 0.0;
          sh.lyy[lane] = lyy[lane];
        }
        if (lane < 14) sh.lx[lane] = lx_l;
        __syncthreads();
        ok = riccati_knot<14, true>(sh, lane, lu, ly, reg, sp.eps9, Kout, duout, Gout, &dV);
      } else {
        if (lane < 10) {
          const double v = nk[lane];
          if (lane < 6) sh.xb[lane] = v;
          else sh.ub[lane - 6] = v;
        }
        __syncthreads();
        double Ac[36], Bc[24];
        srb_jacobians(sh.xb, sh.ub, foot, cs, Ac, Bc);
        for (int e = lane; e < 36 + 24; e += 64) {
          if (e < 36) sh.A[e] = ((e / 6 == e % 6) ? 1.0 : 0.0) + Ac[e] * dt;
          else sh.Bm[e - 36] = Bc[e - 36] * dt;
        }
        const int m = mode - 1;
        double lu[4], ly[4] = {0, 0, 0, 0};
        const double ru[4] = {0, kGRF, 0, kGRF};
        for (int c = 0; c < 4; ++c) lu[c] = (2 * dt * cRfb[m][c]) * (sh.ub[c] - ru[c]);
        double lx_l = 0;
        {
          const int i = lane < 6 ? lane : 0;
          const double rxi = i == 0 ? pos[k] : i == 1 ? sp.height : i == 3 ? sp.vel : 0.0;
          lx_l = (2 * dt * cQfb[i]) * (sh.xb[i] - rxi);
          if (lane < 6) sh.lxx[lane] = 2 * dt * cQfb[lane];
        }
        if (lane < 16) {
          sh.luu[lane] = (lane % 5 == 0) ? 2 * dt * cRfb[m][lane / 5] : 0.0;
          sh.lyy[lane] = 0;
        }
        if (lane < 6) sh.lx[lane] = lx_l;
        __syncthreads();
        ok = riccati_knot<6, false>(sh, lane, lu, ly, reg, sp.eps9, Kout, duout, Gout, &dV);
      }
      ++*knots;
      if (wb) ++*knots_wb;
      if (!ok) {
        st->dV[p] = dV;
        return false;
      }
    }
    st->dV[p] = dV;
  }
  return true;
}

__global__ __launch_bounds__(64) void k_bws(SolveParams sp, DevBufs d, double update_reg) {
  const int b = blockIdx.x;
  if (b >= sp.B) return;
  ProbState* st = &d.st[b];
  if (!(st->active && st->ddp_active)) return;
  __shared__ BwsLds sh;
  double reg = st->reg;
  int bws_iter = 1;
  int64_t knots = 0, knots_wb = 0, px_reads = 0;
  int64_t sweeps = 0;
  bool aborted = false;
  for (;;) {
    ++sweeps;
    const bool ok = bws_sweep(sp, d, b, st, sh, reg, &knots, &knots_wb, &px_reads);
    if (ok) break;
    reg = fmax(reg * update_reg, 1e-03);
    ++bws_iter;
    if (reg > 1000) { aborted = true; break; }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    st->cnt[C_DDP]++;
    st->cnt[C_BWS] += sweeps;
    st->cnt[C_BWS_KNOTS] += knots;
    st->cnt[C_BWS_KNOTS_WB] += knots_wb;
    st->cnt[C_BWS_KNOTS_FB] += knots - knots_wb;
    st->cnt[C_PX_READS] += px_reads;
    st->bws_iter = bws_iter;
    if (aborted) {
      st->status = MHPC_SOLVE_REG_ABORT;
      st->active = 0;
      st->ddp_active = 0;
      if (st->ntrace < TRACE)
        st->trace[st->ntrace++] = (st->al_iter << 24) | (st->reb_active << 23) | (1 << 21) |
                                  (bws_iter & 0xff);
    } else {
      st->dV_exp = st->dV[0];
      reg = reg / 20;
      if (reg < 1e-06) reg = 0;
      st->reg = reg;
    }
  }
}

// ============================================================================================
// AL / ReB update (MultiPhaseDDP.cpp:273-284, SinglePhase.cpp:334-354)
// ============================================================================================
__global__ void k_al_end(SolveParams sp, DevBufs d, int last) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= sp.B) return;
  ProbState* st = &d.st[b];
  if (st->active) {
    double up = sp.update_penalty;
    if (st->viol < 0.03) up = 0;
    for (int p = 0; p < sp.P; ++p) {
      const bool wb = p < sp.n_wb;
      if (ntc_of(sp.mode[p], wb)) st->lambda[p] += st->sigma[p] * st->h[p];
      st->sigma[p] *= up;
      if (st->reb_active && wb) {
        st->delta[p] *= sp.update_relax;
        if (st->delta[p] < 0.01) st->delta[p] = 0.01;
        st->eps_tq[p] *= sp.update_ReB;
        st->eps_grf[p] *= sp.update_ReB;
      }
    }
    if (st->viol < sp.AL_thresh) st->active = 0;
  }
  if (last && st->status == MHPC_SOLVE_OK && !isfinite(st->J)) st->status = MHPC_SOLVE_NONFINITE;
}

// ============================================================================================
// initialization: references, state, PD warm start (MHPCLocomotion.cpp:47-53,200-215)
// ============================================================================================
__global__ void k_init(SolveParams sp, DevBufs d) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= sp.B) return;
  const double* x0 = d.x0 + (size_t)b * 14;
  double* pos = d.refpos + (size_t)b * sp.NK;
  for (int p = 0; p < sp.P; ++p) {
    const int ko = sp.ko[p];
    pos[ko] = p == 0 ? x0[0] : pos[sp.ko[p - 1] + sp.N[p - 1] - 1];
    for (int k = 1; k < sp.N[p]; ++k) pos[ko + k] = pos[ko + k - 1] + sp.vel * sp.dt[p];
  }
  ProbState* st = &d.st[b];
  st->J = 0; st->viol = 0; st->dV_exp = 0; st->reg = 0; st->cost_prev = 0;
  for (int p = 0; p < MAXP; ++p) {
    st->V[p] = 0; st->dV[p] = 0; st->h[p] = 0; st->lambda[p] = 0;
    const bool wb = p < sp.n_wb && p < sp.P;
    st->sigma[p] = (wb && ntc_of(sp.mode[p], true)) ? 5.0 : 0.0;
    st->delta[p] = 0.1;
    st->eps_tq[p] = 0.01;
    st->eps_grf[p] = 0.01;
  }
  st->status = MHPC_SOLVE_OK;
  st->active = 1; st->ddp_active = 0; st->reb_active = 0; st->al_partials = 0;
  st->nom_slot = 0; st->al_iter = 0; st->ddp_iter = 0; st->bws_iter = 0; st->ntrace = 0;
  for (int i = 0; i < TRACE; ++i) st->trace[i] = -1;
  for (int i = 0; i < NCNT; ++i) st->cnt[i] = 0;
  // warm start of the WB phases into slot 0 (bounding_PDcontrol, boundingPDControl.cpp:3-46)
  double x[14];
  for (int i = 0; i < 14; ++i) x[i] = x0[i];
  const double qnom[4] = {PI / 4, -PI * 7 / 12, PI / 4, -PI * 7 / 12};
  const double Kp[4] = {5 * 8.0, 5 * 1.0, 5 * 12.0, 5 * 10.0};
  for (int p = 0; p < sp.n_wb; ++p) {
    const int mode = sp.mode[p], N = sp.N[p], ko = sp.ko[p];
    const double dt = sp.dt[p];
    for (int k = 0; k < N - 1; ++k) {
      double u[4];
      if (mode == 1 || mode == 3) {
        const int foot = mode == 1 ? kBack : kFront;
        double J[14], Jd[14], v[2];
        wb_foot_jacobian(x, foot, J, Jd);
        wb_leg_ext(x, foot, v);
        const double sq = v[0] * v[0] + v[1] * v[1], nrm = sqrt(sq);
        const double n0 = v[0] / nrm, n1 = v[1] / nrm;
        const double F0 = -n0 * 2200.0 * (nrm - 0.2462), F1 = -n1 * 2200.0 * (nrm - 0.2462);
        const double gain = mode == 1 ? 3 : 2.2;
        for (int i = 0; i < 4; ++i) u[i] = (J[3 + i] * F0 + J[7 + 3 + i] * F1) * gain;
      } else {
        for (int i = 0; i < 4; ++i) u[i] = Kp[i] * (qnom[i] - x[3 + i]) - x[10 + i];
      }
      double xd[14], y[4];
      wb_dynamics<double>(x, u, mode, xd, y);
      double* o = traj_ptr(sp, d, b, 0, ko + k);
      for (int i = 0; i < 14; ++i) o[i] = x[i];
      for (int i = 0; i < 4; ++i) { o[14 + i] = u[i]; o[18 + i] = y[i]; }
      for (int i = 0; i < 14; ++i) x[i] = x[i] + xd[i] * dt;
    }
    double* oe = traj_ptr(sp, d, b, 0, ko + N - 1);
    for (int i = 0; i < 14; ++i) oe[i] = x[i];
    if (p + 1 < sp.n_wb && (mode == 2 || mode == 4)) {
      double xp[14], lam[2];
      wb_impact<double>(x, mode == 2 ? kFront : kBack, xp, lam);
      for (int i = 0; i < 14; ++i) x[i] = xp[i];
    }
  }
}

// Copy each problem's nominal trajectory (slot nom_slot) to a dense staging buffer.
__global__ void k_export(SolveParams sp, DevBufs d) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long per = (long)sp.NK * KS;
  const int b = (int)(t / per);
  if (b >= sp.B) return;
  const long r = t - (long)b * per;
  const int nom = d.st[b].nom_slot;
  d.out[(size_t)b * per + r] = d.traj[(((size_t)b * sp.nslot + nom) * sp.NK) * KS + r];
}

// ---- kernel-level parity hooks (batched CasADi replacements) -----------------------------
__global__ void k_eval_wb_dyn(int n, int mode, const double* x, const double* u, double* xd,
                              double* y) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  wb_dynamics<double>(x + (size_t)i * 14, u + (size_t)i * 4, mode, xd + (size_t)i * 14, y + (size_t)i * 4);
}

__global__ void k_eval_wb_par(int n, int mode, const double* x, const double* u, double* Ac,
                              double* Bc, double* C, double* D) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * 18) return;
  const int i = t / 18, dir = t % 18;
  Dual xx[14], uu[4], f[14], y[4];
  for (int a = 0; a < 14; ++a) xx[a] = Dual(x[(size_t)i * 14 + a], a == dir ? 1.0 : 0.0);
  for (int a = 0; a < 4; ++a) uu[a] = Dual(u[(size_t)i * 4 + a], 14 + a == dir ? 1.0 : 0.0);
  wb_dynamics<Dual>(xx, uu, mode, f, y);
  if (dir < 14) {
    for (int r = 0; r < 14; ++r) Ac[(size_t)i * 196 + r * 14 + dir] = f[r].d;
    for (int r = 0; r < 4; ++r) C[(size_t)i * 56 + r * 14 + dir] = y[r].d;
  } else {
    for (int r = 0; r < 14; ++r) Bc[(size_t)i * 56 + r * 4 + dir - 14] = f[r].d;
    for (int r = 0; r < 4; ++r) D[(size_t)i * 16 + r * 4 + dir - 14] = y[r].d;
  }
}

__global__ void k_eval_wb_impact(int n, int foot, const double* x, double* xp, double* Px) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * 14) return;
  const int i = t / 14, dir = t % 14;
  Dual xx[14], yy[14], lam[2];
  for (int a = 0; a < 14; ++a) xx[a] = Dual(x[(size_t)i * 14 + a], a == dir ? 1.0 : 0.0);
  wb_impact<Dual>(xx, foot, yy, lam);
  for (int r = 0; r < 14; ++r) Px[(size_t)i * 196 + r * 14 + dir] = yy[r].d;
  if (dir == 0)
    for (int r = 0; r < 14; ++r) xp[(size_t)i * 14 + r] = yy[r].v;
}

__global__ void k_eval_srb(int n, const double* x, const double* u, const double* p,
                           const double* s, double* xd, double* Ac, double* Bc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  srb_dynamics(x + (size_t)i * 6, u + (size_t)i * 4, p + (size_t)i * 4, s + (size_t)i * 2, xd + (size_t)i * 6);
  srb_jacobians(x + (size_t)i * 6, u + (size_t)i * 4, p + (size_t)i * 4, s + (size_t)i * 2, Ac + (size_t)i * 36, Bc + (size_t)i * 24);
}

// Sum the per-problem counters of the batch (int64 atomics into NCNT slots).
__global__ void k_reduce_counters(SolveParams sp, DevBufs d, unsigned long long* out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= sp.B) return;
  for (int i = 0; i < NCNT; ++i) atomicAdd(&out[i], (unsigned long long)d.st[b].cnt[i]);
}

// ---- launchers (called by mhpc_runtime.cpp) ---------------------------------------------
hipError_t launch_reduce_counters(const SolveParams& sp, const DevBufs& d,
                                  unsigned long long* out, hipStream_t s) {
  hipLaunchKernelGGL(k_reduce_counters, dim3((sp.B + 255) / 256), dim3(256), 0, s, sp, d, out);
  return hipGetLastError();
}
hipError_t launch_init(const SolveParams& sp, const DevBufs& d, hipStream_t s) {
  hipLaunchKernelGGL(k_init, dim3((sp.B + 63) / 64), dim3(64), 0, s, sp, d);
  return hipGetLastError();
}
hipError_t launch_rollout(const SolveParams& sp, const DevBufs& d, int full, int al_iter,
                          int ddp_iter, int max_ddp, hipStream_t s) {
  const int nc = full ? 1 : sp.n_cand;
  const int ppw = 64 / nc;
  hipLaunchKernelGGL(k_rollout, dim3((sp.B + ppw - 1) / ppw), dim3(64), 0, s, sp, d, full,
                     al_iter, ddp_iter, max_ddp);
  return hipGetLastError();
}
hipError_t launch_partials(const SolveParams& sp, const DevBufs& d, hipStream_t s) {
  const long total = (long)sp.B * sp.par_items;
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(k_partials, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, sp, d);
  return hipGetLastError();
}
hipError_t launch_bws(const SolveParams& sp, const DevBufs& d, double update_reg, hipStream_t s) {
  hipLaunchKernelGGL(k_bws, dim3(sp.B), dim3(64), 0, s, sp, d, update_reg);
  return hipGetLastError();
}
hipError_t launch_al_end(const SolveParams& sp, const DevBufs& d, int last, hipStream_t s) {
  hipLaunchKernelGGL(k_al_end, dim3((sp.B + 63) / 64), dim3(64), 0, s, sp, d, last);
  return hipGetLastError();
}
hipError_t launch_export(const SolveParams& sp, const DevBufs& d, hipStream_t s) {
  const long total = (long)sp.B * sp.NK * KS;
  hipLaunchKernelGGL(k_export, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, sp, d);
  return hipGetLastError();
}
hipError_t launch_eval_wb_dyn(int n, int mode, const double* x, const double* u, double* xd,
                              double* y, hipStream_t s) {
  hipLaunchKernelGGL(k_eval_wb_dyn, dim3((n + 63) / 64), dim3(64), 0, s, n, mode, x, u, xd, y);
  return hipGetLastError();
}
hipError_t launch_eval_wb_par(int n, int mode, const double* x, const double* u, double* Ac,
                              double* Bc, double* C, double* D, hipStream_t s) {
  hipLaunchKernelGGL(k_eval_wb_par, dim3((n * 18 + 63) / 64), dim3(64), 0, s, n, mode, x, u, Ac,
                     Bc, C, D);
  return hipGetLastError();
}
hipError_t launch_eval_wb_impact(int n, int foot, const double* x, double* xp, double* Px,
                                 hipStream_t s) {
  hipLaunchKernelGGL(k_eval_wb_impact, dim3((n * 14 + 63) / 64), dim3(64), 0, s, n, foot, x, xp, Px);
  return hipGetLastError();
}
hipError_t launch_eval_srb(int n, const double* x, const double* u, const double* p,
                           const double* c, double* xd, double* Ac, double* Bc, hipStream_t s) {
  hipLaunchKernelGGL(k_eval_srb, dim3((n + 63) / 64), dim3(64), 0, s, n, x, u, p, c, xd, Ac, Bc);
  return hipGetLastError();
}

}  // namespace mhpc
