// Device-side data model of the batched HSDDP solve (shared by kernels and runtime).
//
// HBM layout (one handle = one batch of B problems; each problem has its own phase layout --
// gait schedule -- drawn from the handle's layout table, and problems sharing a layout form a
// group; every array is problem-major so each problem's records are contiguous and a wave's
// loads of one knot record are coalesced):
//   traj   [B][NSLOT][NK][KS]  x(<=14) u(4) y(4) per knot, KS = 24 doubles.  NSLOT =
//          n_cand + 1 rollout slots; state.nom_slot names the nominal trajectory and the
//          line-search candidates write the other slots (no copy on acceptance).  NK is the
//          per-problem knot stride: the largest knot count of the handle's layouts.
//   refpos [B][NK]             forward position reference (ReferenceGen.h:94-109); the
//          rest of the reference is constant per mode and computed in registers.
//   K      [B][NK][56], du [B][NK][4], G [B][NK][14]   CostToGoStruct outputs per knot.
//   par    [B][18][NK][9] + [B][NK][14] (NK * PS per problem, par_col / par_jac below)
//          dynamics Jacobians of the nominal trajectory: 18 tangent directions x (7 qddot
//          rows + 2 contact-force rows) per WB knot, column-block major, then the knots'
//          control/force cost derivatives incl. the ReB barrier (computed once per partials
//          pass, so the backward kernel evaluates no transcendental); SRB knots are
//          differentiated in registers by the backward kernel.
//   px     [B][P][196]         impact Jacobian Px (column-major) at the end of WB phases.
//   state  [B]                 ProbState (control flow + AL/ReB parameters).
//   lay    [L]                 Layout table (read through the constant address space: scalar
//          loads), gidx [B] the problems grouped by layout (group g = positions
//          [go[g], go[g+1]) of gidx), lid [B] each problem's layout.
#pragma once
#include <stdint.h>

#include "mhpc_real.h"

#include "../../include/mhpc_capi.h"

namespace MHPC_NS {

constexpr int KS = 24;        // doubles per knot record in traj
constexpr int PS_JAC = 162;   // 18 tangent directions x (7 qddot + 2 contact-force rows)
constexpr int PS = 176;       // doubles per knot in par: Jacobians + 14 cost derivatives
                              // (lu 4, luu 4, ly 2, lyy 4 of the stance block)
// par, per problem (NK = the knot stride, sp.NK): 18 column blocks [NK][9] -- column c of
// knot k at (c NK + k) 9 -- then the cost derivatives [NK][14].  A direction's values of
// consecutive knots are contiguous, so the partials' lanes (consecutive knots) store whole
// lines; the sweep's lane walks its own column block backwards, one 72-byte piece per knot.
__host__ __device__ inline size_t par_col(int NK, int b, int c, int kk) {
  return (size_t)b * NK * PS + ((size_t)c * NK + kk) * 9;
}
__host__ __device__ inline size_t par_jac(int NK, int b, int kk) {
  return (size_t)b * NK * PS + (size_t)PS_JAC * NK + (size_t)kk * 14;
}
constexpr int MAXP = MHPC_MAX_PHASES;
constexpr int MAXC = 32;      // max line-search candidates
constexpr int MAXL = MHPC_MAX_LAYOUTS;  // distinct phase layouts per handle
constexpr int ST_RMAX = 128;  // line search: staged position references per problem (knots per phase)
constexpr int TRACE = MHPC_TRACE_LEN;

// Counter slots of ProbState::cnt.  C_LS is the reference-equivalent number of serial
// line-search rollouts; C_*_RUN count what this implementation actually executed; the
// knot / Px counters feed the algorithmic-byte model of the roofline report.
enum {
  C_DDP = 0, C_BWS, C_BWS_KNOTS, C_LS, C_FWD, C_PAR, C_LS_RUN, C_PAR_RUN,
  C_LS_LAUNCH, C_BWS_KNOTS_WB, C_BWS_KNOTS_FB, C_PX_READS,
  C_BWS_KNOTS_FB1,  // SRB knots swept by the SRB half of a split sweep (its first attempt)
  NCNT
};

struct CostParams {
  real wQ[4][14], wR[4][4], wS[4][4], wQf[4][14];  // whole-body phases
  real fQ[4][6], fR[4][4], fQf[4][6];              // SRB phases
  real tq_lim, mu;                                 // torque limit, GRF friction coefficient
  real sigma0[4], delta0[4], delta_min[4], eps_tq0[4], eps_grf0[4];  // AL / ReB initial values
};

// Phase layout of one group of problems (MHPCLocomotion::build_problem, MHPCLocomotion.cpp
// :63-104, for that problem's gait point): n_wb whole-body phases, then SRB phases.
struct Layout {
  int P, n_wb, NK;          // phases, whole-body phases, knots of this layout (<= SolveParams::NK)
  int mode[MAXP], N[MAXP], ko[MAXP], xs[MAXP];
  int buf[MAXP];            // phase buffer of each phase (receding horizon, see k_store_*)
  // partials work per problem and its prefix offsets per phase: WB knots with Jacobians
  // (N - 1 per WB phase) and impact directions (14 per touchdown phase)
  int par_knots, par_imp;
  int par_knot_off[MAXP + 1], par_imp_off[MAXP + 1];
  real dt[MAXP];
};

struct SolveParams {
  int B;                   // problems of the handle (the arrays' leading dimension)
  int NK;                  // per-problem knot stride of the packed arrays (max over layouts)
  // layout groups: the problems of group g are gidx[go[g] .. go[g + 1]) and share layout g;
  // a launch enumerates its blocks group by group, so no block mixes layouts (kernels map a
  // block to its group with block_group, mhpc_device.h).  ident: gidx is the identity.
  int ngrp, ident;
  int go[MAXL + 1];
  int gpk[MAXL], gpi[MAXL];  // partials knot / impact work items per problem of each group
  int pmax;                  // most phases of any layout
  real vel, height;
  int n_cand, nslot;
  real eps[MAXC];          // line-search grid 1, alpha, alpha^2, ... (host libm)
  real gamma, DDP_thresh, AL_thresh, update_penalty, update_relax, update_regularization,
      update_ReB;
  real eps9;               // pow(0.1, 9) (SinglePhase.cpp:202), host libm
  int AL_active, ReB_active;
  // launch shape (host side only): compute units of the handle's device and the kernel
  // variants forced through mhpc_set_kernel_variant (0 = chosen by batch size)
  int ncu, var_bws, var_ro, var_overlap;
  // line-search trials that store their running knot records (the first ro_store, and the
  // last; the rest are rolled out again when accepted -- mhpc_kernels.hip RO_STORE_FIRST)
  int ro_store;
  // host side: some layout has both kinds of phase (the sweep can run split, bws_split) /
  // every phase of every layout fits the line search's LDS stage of position references
  int split_ok, stage_fits;
  // cost weights (diagonals per mode, CostBase.h:9-46 / MHPCCost.cpp:24-75) and constraint
  // parameters (ConstraintsBase.h:11-50 / MHPCConstraints.cpp:14-88): mhpc_set_cost_weights /
  // mhpc_set_constraint_params; read by every kernel from its parameter block
  CostParams cw;
};

// Costs, their sums and the expected cost change are accumulated and compared in fp64 in
// both builds (the fp32 build keeps its dynamics, partials and sweep in fp32): a total cost
// of ~1e5 summed over ~700 knots in fp32 carries errors of the size of the Armijo margins.
using acc = double;

struct ProbState {
  acc J, viol, dV_exp;
  real reg;
  acc cost_prev;
  acc V[MAXP], dV[MAXP];
  real h[MAXP];
  real sigma[MAXP], lambda[MAXP], delta[MAXP], eps_tq[MAXP], eps_grf[MAXP];
  int32_t status;      // mhpc_solve_status
  int32_t active;      // still inside the AL loop
  int32_t ddp_active;  // still inside the DDP loop of this AL iteration
  int32_t reb_active;  // _option.ReB_active of this AL iteration
  int32_t al_partials; // terminal AL partials present (B1: only after forward_sweep(0))
  int32_t nom_slot;
  int32_t al_iter, ddp_iter;
  int32_t bws_iter;    // backward sweeps of this DDP iteration
  int32_t ntrace;
  int32_t trace[TRACE];
  int64_t cnt[NCNT];
  // state of the last running/terminal-cost partials evaluation (forward_sweep(0) or
  // forward_sweep_partials_only) for print_debugInfo's cost.txt: the nominal slot it saw,
  // whether the AL terms entered Phix (B1) and the sigma / lambda it used
  int32_t par_slot, par_al;
  real par_sigma[MAXP], par_lambda[MAXP];
  // line-search trials run after that evaluation (only the final, converged line search of
  // an AL iteration): the reference's dynamics-only sweeps add their AL terms to Phix too
  // (guard quirk of SinglePhase.cpp:269), which cost.txt shows.  Trial j lives in slot
  // j < ls_nom ? j : j + 1.
  int32_t ls_nt, ls_nom;
  real ls_sigma[MAXP], ls_lambda[MAXP];
  // line-search trial whose running records were not stored (trials j >= RO_STORE_FIRST but
  // the last, mhpc_kernels.hip) and must be rolled out again into its slot, -1 if none; the
  // nominal slot that line search started from
  int32_t reroll_j, reroll_nom;
  real reroll_eps;  // its step size (eps of trial reroll_j)
  // MultiPhaseDDP::_option as solve() leaves it: ReB_active and update_penalty are rewritten
  // inside the AL loop (MultiPhaseDDP.cpp:178-183, 273-277) and the next solve() starts from
  // the rewritten values (captured at its first AL iteration: cap_*) -- visible across the
  // solves of a receding-horizon loop.  mhpc_initialize restores the handle's options.
  int32_t opt_reb, cap_reb;
  real opt_pen, cap_pen;
};

// Value function where the backward sweep crosses from the SRB phases into the WB phases
// (the sweep runs as two launches when the SRB part overlaps the partials):
// H / G of knot 0 of phase n_wb (row stride NX of that phase) from the first attempt whose
// SRB part passed the PSD test -- the SRB half retries attempts that fail there itself --,
// that attempt's regularisation and number (bws_iter), whether the retries aborted
// (regularisation > 1000), the attempts and SRB knots swept.
struct BwsCarry {  // double in both builds: the sweep's arithmetic type (mhpc_bws.hip breal)
  double H[196];
  double G[14];
  double reg;
  int32_t abort, iter, sweeps, knots;
};

struct DevBufs {
  real* traj;
  real* refpos;
  real* K;
  real* du;
  real* G;
  real* par;
  real* px;
  real* x0;
  ProbState* st;
  real* out;    // export staging [B][NK][KS]
  BwsCarry* carry;  // [B]
  const Layout* lay;  // [ngrp] layout table
  const int* gidx;    // [B] problems grouped by layout
  const int* lid;     // [B] layout of each problem
};

}  // namespace MHPC_NS
