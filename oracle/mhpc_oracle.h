/* TEST INFRASTRUCTURE ONLY.  C ABI of the CPU oracle (oracle/hsddp_oracle.cpp): a
 * line-faithful restatement of the reference HSDDP solve (no Eigen) whose dynamics are the
 * reference's own CasADi kernels (oracle/_ref).  Used by tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg -- never by the product library. */
#ifndef MHPC_ORACLE_H
#define MHPC_ORACLE_H
#include <stdint.h>
#include "../include/mhpc_capi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Load the CasADi reference kernels from `path` (oracle/_ref/libmhpc_casadi_ref.so). */
int oracle_load_ref(const char* path);

/* Cost weights / constraint parameters for later calls (counterpart of
 * mhpc_set_cost_weights / mhpc_set_constraint_params); NULL = the reference's values. */
int oracle_set_params(const mhpc_cost_weights* w, const mhpc_constraint_params* c);

/* Solve `batch` independent problems (x0: [batch][xsize of phase 0]).
 * do_solve = 0 runs initialization only (refs + PD warm start), leaving the nominal
 * trajectory of the warm start in the outputs.
 * Per-problem outputs are phase-concatenated (phase 0 knots, then phase 1 ...):
 *   X [batch][sum_p N_p*n_p], U,Y,DU [batch][sum_p N_p*4], K [batch][sum_p N_p*4*n_p],
 *   G [batch][sum_p N_p*n_p]; J, dV, viol [batch]; Vp, dVp [batch][n_phases];
 *   status [batch]; trace [batch][MHPC_TRACE_LEN];
 *   counters [batch][6] = ddp_iters, bws_sweeps, bws_knots, ls_rollouts, fwd_sweeps,
 *   partial_sweeps.  Any output pointer may be NULL. */
int oracle_solve(const mhpc_problem_desc* desc, const mhpc_hsddp_option* opt, int batch,
                 const double* x0, int nthreads, int do_solve, double* X, double* U, double* Y,
                 double* K, double* DU, double* G, double* J, double* dV, double* viol,
                 double* Vp, double* dVp, int32_t* status, int32_t* trace, int64_t* counters);

#ifdef __cplusplus
}
#endif
#endif
