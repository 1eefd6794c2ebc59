/* mhpc_capi.h -- C-ABI boundary of the MI355X-native HSDDP solve path.
 *
 * Drop-in for the solve path that the reference runs under
 * MHPCLocomotion<double>::solve_mhpc() (Controller/MHPCLocomotion/MHPCLocomotion.cpp:167-195
 * -> HSDDPSolver/source/MultiPhaseDDP.cpp:154-289).  Plain C types only: pointers, sizes,
 * POD structs; no exceptions cross the ABI; every entry point returns an mhpc_status
 * (0 = OK).  One handle owns the device-resident state of a BATCH of independent MPC
 * problems; each problem has its own phase layout (gait schedule) drawn from a table of up to
 * MHPC_MAX_LAYOUTS distinct layouts (mhpc_set_layouts; by default every problem has the
 * layout given at create).  Calls on one handle are serialised by the caller; different
 * handles (devices, streams) are independent.
 *
 * Reference interfaces replaced (file:line in /root/reference):
 *   mhpc_create          MHPCLocomotion ctor + memory_alloc      (MHPCLocomotion.cpp:8-43,218-261)
 *   mhpc_set_x0          MultiPhaseDDP::set_initial_condition   (MultiPhaseDDP.h:24-25); the
 *                        reference overwrites _x0 with its private default in
 *                        initialization() (MHPCLocomotion.cpp:49) -- settable here so a batch can
 *                        carry random initial states
 *   mhpc_initialize      MHPCLocomotion::initialization         (MHPCLocomotion.cpp:47-53):
 *                        memory_reset + build_problem (ReferenceGen::generate_ref,
 *                        ReferenceGen.h:53-109) + warmstart (bounding_PDcontrol,
 *                        boundingPDControl.cpp:3-46)
 *   mhpc_solve           MHPCLocomotion::solve_mhpc / MultiPhaseDDP::solve
 *                        (MHPCLocomotion.cpp:167-195, MultiPhaseDDP.cpp:154-289)
 *   mhpc_get_phase       SinglePhase::get_nominal_ms_ptr / get_CTG_info_ptr
 *                        (SinglePhase.cpp:364-373; fields of ModelState / CostToGoStruct,
 *                        MHPC_CompoundTypes.h:7-22,88-145)
 *   mhpc_get_scalars     MultiPhaseDDP::_actual_cost / _exp_cost_change /
 *                        _tconstr_violation and SinglePhaseAbstract::_V/_dV
 *                        (MultiPhaseDDP.h:57-60, SinglePhaseAbstract.h:116-118)
 *   mhpc_destroy         MHPCLocomotion::~MHPCLocomotion / memory_free (MHPCLocomotion.cpp:383-470)
 *   mhpc_update_problem  MHPCLocomotion::update_problem          (MHPCLocomotion.cpp:107-158,
 *                        Gait.h:21-77): gait advance, phase-buffer rotation, re-init
 *   mhpc_set_layouts     one MHPCLocomotion per controller, each built from its own Gait
 *                        (MHPCLocomotion.cpp:63-104): per-problem phase layouts in one batch
 *   mhpc_update_problems update_problem of every controller with its own gait and step count
 */
#ifndef MHPC_CAPI_H
#define MHPC_CAPI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MHPC_MAX_PHASES 16
#define MHPC_MAX_KNOTS 1024
#define MHPC_MAX_LAYOUTS 32   /* distinct phase layouts (gait schedules) per handle */
#define MHPC_TRACE_LEN 64

typedef enum {
  MHPC_OK = 0,
  MHPC_ERR_INVALID = 1,  /* bad argument / descriptor */
  MHPC_ERR_DEVICE = 2,   /* HIP runtime error (message via mhpc_last_error) */
  MHPC_ERR_STATE = 3     /* call order violated (e.g. solve before initialize) */
} mhpc_status;

/* Per-problem solve outcome (status array of mhpc_solve). */
typedef enum {
  MHPC_SOLVE_OK = 0,          /* finished all AL iterations or met AL_thresh */
  MHPC_SOLVE_REG_ABORT = 1,   /* regularization > 1000: early return (MultiPhaseDDP.cpp:218-226) */
  MHPC_SOLVE_NONFINITE = 2    /* non-finite total cost at the end of the solve */
} mhpc_solve_status;

/* Phase layout. As in MHPCLocomotion::build_problem (MHPCLocomotion.cpp:63-104) the n_wb
 * whole-body phases come first, then n_fb single-rigid-body phases; mode_seq[p] in 1..4
 * (1 back stance, 2 flight, 3 front stance, 4 flight); N[p] knots per phase.  dt values
 * are the reference's float parameters promoted to double.
 * n_wb == 0 is accepted (SRB-only problems, config C1). */
typedef struct {
  int32_t n_wb;
  int32_t n_fb;
  int32_t mode_seq[MHPC_MAX_PHASES];
  int32_t N[MHPC_MAX_PHASES];
  double dt_wb;
  double dt_fb;
  double vel_cmd;     /* USRCMD::vel (float promoted) */
  double height_cmd;  /* USRCMD::height */
  int32_t precision;  /* 64: fp64 (the reference's MHPCLocomotion<double>); 32: the fp32
                       * instantiation of the same kernels (config C5).  Host arrays at
                       * the ABI stay double in both cases. */
  int32_t reserved;
} mhpc_problem_desc;

/* Field-for-field HSDDP_OPTION<double> (MHPC_CompoundTypes.h:196-212). */
typedef struct {
  double alpha;
  double gamma;
  double update_penalty;
  double update_relax;
  double update_regularization;
  double update_ReB;
  double max_DDP_iter;
  double max_AL_iter;
  double DDP_thresh;
  double AL_thresh;
  int32_t AL_active;
  int32_t ReB_active;
  int32_t smooth_active;
  int32_t reserved;
} mhpc_hsddp_option;

/* Aggregate counters of the last mhpc_solve (sums over the batch). */
typedef struct {
  int64_t ddp_iters;        /* inner DDP iterations executed */
  int64_t bws_sweeps;       /* backward sweeps incl. failed (retried) ones */
  int64_t bws_knots;        /* knots swept backward (incl. partial failed sweeps) */
  int64_t ls_rollouts;      /* line-search rollouts the serial reference would run */
  int64_t fwd_sweeps;       /* full forward sweeps (forward_sweep(0)) */
  int64_t partial_sweeps;   /* forward_sweep_partials_only calls */
  double solve_ms;          /* device time of the last solve (HIP events) */
} mhpc_counters;

typedef struct mhpc_handle mhpc_handle;

/* Library identification / diagnostics. */
const char* mhpc_version(void);
const char* mhpc_last_error(void);

/* Number of knots/entries helpers for sizing caller buffers. */
int mhpc_phase_dims(const mhpc_problem_desc* desc, int phase, int* xsize, int* N);

int mhpc_create(const mhpc_problem_desc* desc, const mhpc_hsddp_option* opt, int batch,
                int device, mhpc_handle** out);
/* x0: [batch][xsize of phase 0] row-major host array. */
int mhpc_set_x0(mhpc_handle* h, const double* x0);
int mhpc_initialize(mhpc_handle* h);
/* status: optional host array [batch] of mhpc_solve_status. */
int mhpc_solve(mhpc_handle* h, int32_t* status);
/* Copy out the nominal solution of one phase; any pointer may be NULL.
 * Shapes (row-major, host): x [batch][N][xsize], u/y/du [batch][N][4],
 * K [batch][N][4][xsize], Vx [batch][N][xsize]. */
int mhpc_get_phase(mhpc_handle* h, int phase, double* x, double* u, double* y, double* K,
                   double* du, double* Vx);
/* mhpc_get_phase for problems [first, first + count) of the batch only (shapes with
 * count in place of batch): one problem's phase, as the reference's single-problem
 * _phases[p]->get_nominal_ms_ptr() / get_CTG_info_ptr() hold it (SinglePhaseAbstract.h:79-81). */
int mhpc_get_phase_problems(mhpc_handle* h, int phase, int first, int count, double* x, double* u,
                            double* y, double* K, double* du, double* Vx);
/* J, dV_exp, viol: [batch]; V_phase, dV_phase: [batch][P] with P = mhpc_max_phases (the
 * largest phase count over the problems' layouts -- not mhpc_get_desc's n_wb + n_fb, which is
 * problem 0's; entries past a problem's own phases are zero); trace: [batch][MHPC_TRACE_LEN]
 * (decision trace, encoding in DESIGN.md §Parity); any pointer may be NULL. */
int mhpc_get_scalars(mhpc_handle* h, double* J, double* dV_exp, double* viol, double* V_phase,
                     double* dV_phase, int32_t* trace);
int mhpc_get_counters(mhpc_handle* h, mhpc_counters* c);

/* Gait schedule (the reference's Gait class, Common/header/Gait.h:14-77): the mode cycle and
 * the duration of every mode (timings[m-1], float as in the reference). */
typedef struct {
  int n_modes;
  int modes[MHPC_MAX_PHASES];
  float timings[MHPC_MAX_PHASES];
} mhpc_gait;

/* MHPCLocomotion::update_problem (MHPCLocomotion.cpp:107-158), whole batch: advance the gait
 * by one mode, rotate the WB / SRB phase buffers by one (the solution just computed becomes
 * the warm start of the shifted horizon), recompute mode sequence and knot counts
 * (round(timing / dt)), regenerate the references from the current x0 (set it first with
 * mhpc_set_x0 -- the reference's set_initial_condition) and re-initialise the AL / ReB
 * parameters.  Then call mhpc_solve again.  The phase descriptor reported by
 * mhpc_get_desc changes accordingly. */
int mhpc_update_problem(mhpc_handle* h, const mhpc_gait* gait);
/* The handle's current phase layout (changes with mhpc_update_problem); with per-problem
 * layouts (mhpc_set_layouts) the layout of problem 0. */
int mhpc_get_desc(mhpc_handle* h, mhpc_problem_desc* desc);

/* ---- per-problem phase layouts: the batch axis over gait schedules --------------------
 * In the reference every controller instance builds its phase layout from its own Gait and
 * gait point (MHPCLocomotion::build_problem, MHPCLocomotion.cpp:63-104; Gait.h:21-77) and
 * rotates it per control tick (update_problem, :107-158).  A handle starts with the
 * descriptor of mhpc_create for every problem; mhpc_set_layouts gives problem b the
 * descriptor descs[layout_of_problem[b]] (1 <= n_desc <= MHPC_MAX_LAYOUTS; precision,
 * vel_cmd and height_cmd must equal the handle's; NULL layout_of_problem: descs[b % n_desc]).
 * The arrays grow when a layout has more knots than any before.  The handle is then
 * uninitialised: mhpc_set_x0 (rows of 14 when any layout has a whole-body phase -- an
 * SRB-only problem reads the first 6 of its row -- else 6) and mhpc_initialize precede the
 * next solve.  Problems sharing a layout are solved together, a launch never mixes layouts
 * inside a block, and each problem's arithmetic is the one it gets in a handle of its own
 * layout, bit for bit (tests/test_gpu_layouts.py).  Outputs: mhpc_get_phase_problems needs
 * a problem range whose phase has one shape (knots, state size); mhpc_get_scalars' V_phase /
 * dV_phase rows are max-phase-count long, zero past a problem's phases. */
int mhpc_set_layouts(mhpc_handle* h, int n_desc, const mhpc_problem_desc* descs,
                     const int32_t* layout_of_problem);
/* The current phase layout of problem b (changes with mhpc_update_problem[s]). */
int mhpc_get_problem_desc(mhpc_handle* h, int problem, mhpc_problem_desc* desc);
/* Per-problem MHPCLocomotion::update_problem: problem b takes steps[b] >= 0 gait steps of
 * gaits[gait_of_problem[b]] (one step = one update_problem: the WB / SRB phase buffers
 * rotate by one, the next mode starts the horizon, knot counts round(timing / dt)); with
 * steps[b] = 0 it keeps its layout and warm start.  Every problem's references are then
 * regenerated from its current x0 and its AL / ReB parameters re-initialised, as
 * update_problem does, and the next mhpc_solve starts from the (rotated) solutions.
 * NULL gait_of_problem: gaits[0] for every problem; NULL steps: one step each (then this is
 * mhpc_update_problem).  n_gaits in 1..MHPC_MAX_LAYOUTS. */
int mhpc_update_problems(mhpc_handle* h, int n_gaits, const mhpc_gait* gaits,
                         const int32_t* gait_of_problem, const int32_t* steps);
/* Distinct phase layouts currently in use (1 for a homogeneous batch). */
int mhpc_num_layouts(mhpc_handle* h, int* n);
/* The largest phase count over the problems' current layouts: the row length of
 * mhpc_get_scalars' V_phase / dV_phase. */
int mhpc_max_phases(mhpc_handle* h, int* n);

/* ---- cost and constraint parameters (the reference's downward plugin points) --------
 * The reference's solve reads its weights through CostAbstract / Cost<T,X,U,Y>
 * (HSDDPSolver/header/CostBase.h:9-46: diagonal _Q, _R, _S, _Qf per mode) and its
 * inequality / AL parameters through Constraint (ConstraintsBase.h:11-50: AL_REB_PARAMETER per
 * mode), with the values MHPCCost.cpp:24-75 and MHPCConstraints.cpp:14-88 set.  A handle
 * starts from those values; mhpc_set_* replaces them for every later solve (they travel in
 * the kernels' parameter block).  Rows are modes 1..4. */
typedef struct {
  double wb_Q[4][14];  /* WBCost _Q diagonal (0.01 * q) */
  double wb_R[4][4];   /* WBCost _R diagonal (0.5 * r[m]) */
  double wb_S[4][4];   /* WBCost _S diagonal (s[m]; s[3] uninitialised in the reference: 0) */
  double wb_Qf[4][14]; /* WBCost _Qf diagonal (100 * qf[m]) */
  double fb_Q[4][6];   /* FBCost _Q diagonal (0.01 * q) */
  double fb_R[4][4];   /* FBCost _R diagonal (r[m]); FBCost _S is zero (SRB y == 0) */
  double fb_Qf[4][6];  /* FBCost _Qf diagonal (100 * qf) */
} mhpc_cost_weights;

typedef struct {
  double torque_limit;     /* WBConstraint b_torque: -limit <= u_i <= limit (33) */
  double friction_coeff;   /* WBConstraint _friccoeff of the GRF cone (0.5) */
  double sigma[4];         /* AL penalty at initialisation, modes with a touchdown
                              constraint (2, 4) only: 5 */
  double delta[4];         /* ReB relaxation at initialisation (0.1) */
  double delta_min[4];     /* its lower bound in the AL update (0.01) */
  double eps_torque[4];    /* ReB weight of the torque limits (0.01) */
  double eps_grf[4];       /* ReB weight of the GRF constraints, stance modes 1 / 3 (0.01) */
  /* The joint limits carry eps_ReB = 0 in the reference (MHPCConstraints.cpp:60-82) and
   * contribute exact zeros; they are not a parameter here. */
} mhpc_constraint_params;

/* The reference's values (MHPCCost.cpp:24-75, MHPCConstraints.cpp:14-88). */
int mhpc_default_cost_weights(mhpc_cost_weights* w);
int mhpc_default_constraint_params(mhpc_constraint_params* c);
/* Replace / read the handle's parameters; take effect from the next mhpc_initialize /
 * mhpc_update_problem (AL / ReB initial values) and mhpc_solve (weights, limits).  Every
 * entry must be finite, weights >= 0, torque_limit > 0, friction_coeff >= 0,
 * 0 < delta_min <= delta.  Constraint parameters set on an initialized handle make
 * mhpc_solve return MHPC_ERR_STATE until mhpc_initialize or mhpc_update_problem has applied
 * their initial values (a solve would otherwise run the new limits with the old AL / ReB
 * state). */
int mhpc_set_cost_weights(mhpc_handle* h, const mhpc_cost_weights* w);
int mhpc_get_cost_weights(mhpc_handle* h, mhpc_cost_weights* w);
int mhpc_set_constraint_params(mhpc_handle* h, const mhpc_constraint_params* c);
int mhpc_get_constraint_params(mhpc_handle* h, mhpc_constraint_params* c);

/* Running-cost gradient lx of knots 0..N-2 ([batch][N-1][n]) and terminal-cost gradient Phix
 * ([batch][n]) of `phase` as the last partials evaluation left them: the reference's
 * rcost_*[p][k].lx and tcost_*[p].Phix that print_debugInfo writes to cost.txt
 * (MHPCLocomotion.cpp:355-377; AL terms in Phix only after forward_sweep(0), quirk B1).
 * Either pointer may be NULL. */
int mhpc_get_cost_gradients(mhpc_handle* h, int phase, double* lx, double* Phix);
/* The same for problems [first, first + count) (rows of count in place of batch); with
 * per-problem layouts the range's phase must have one shape. */
int mhpc_get_cost_gradients_problems(mhpc_handle* h, int phase, int first, int count, double* lx,
                                     double* Phix);

/* The trial rollouts of MultiPhaseDDP::forward_iteration (MultiPhaseDDP.cpp:130-151, i.e.
 * SinglePhase::forward_sweep_dynamics_only, SinglePhase.cpp:117-144, chained over phases by
 * MultiPhaseDDP::forward_sweep_dynamics_only :56-76) at n_eps arbitrary step sizes, from the
 * handle's current nominal, gains and AL/ReB state (after mhpc_solve, or right after
 * mhpc_initialize), costs only, nothing modified: J = actual cost, viol = terminal-
 * constraint violation, both [batch][n_eps].  ms (optional) = device time of the launch.
 * The C2 workload (256 concurrent rollouts of one nominal). */
#define MHPC_MAX_ROLLOUT_EPS 4096
int mhpc_rollout_costs(mhpc_handle* h, int n_eps, const double* eps, double* J, double* viol,
                       float* ms);

/* Per-kernel device timing (HIP events around every launch on the handle's stream) and the
 * algorithmic HBM bytes each kernel must move (model in DESIGN.md §Roofline), accumulated
 * over all solves since the last reset.  Kernel ids: 0 init, 1 forward_sweep(0) cost,
 * 2 line search (rollouts + costs + selection), 3 partials, 4 backward_sweep (whole, or its
 * WB half when split), 5 al_update, 6 the SRB half of a split backward sweep. */
#define MHPC_NUM_KERNELS 7
const char* mhpc_kernel_name(int k);
int mhpc_set_profiling(mhpc_handle* h, int on);
int mhpc_get_kernel_stats(mhpc_handle* h, double* ms, int64_t* launches, double* alg_bytes);
int mhpc_reset_kernel_stats(mhpc_handle* h);
/* Algorithmic FP64 flops per kernel accumulated like mhpc_get_kernel_stats' bytes: the
 * backward sweep in the reference's dense formulation; 0 for the others. */
int mhpc_get_kernel_flops(mhpc_handle* h, double* flops);
void mhpc_destroy(mhpc_handle* h);

/* Kernel variants.  The launch shape of the backward sweep and of the line search is chosen
 * from the batch size and the device's compute-unit count; every variant
 * computes the same per-problem arithmetic, bit for bit (tests/test_gpu_variants.py).  This
 * call pins one variant for the handle's later solves -- for parity tests of every variant
 * at any batch size, and for tuning.  variant 0 restores the automatic choice.
 * MHPC_ERR_INVALID if the variant does not apply (the staged line-search variants need at
 * least 10 line-search candidates, the pair variant at most 32). */
#define MHPC_VARIANT_BWS 0            /* which: backward sweep */
#define MHPC_VARIANT_BWS_ROWS4 1      /*   four problems per wave (one per 16-lane row) */
#define MHPC_VARIANT_BWS_ROWS2 2      /*   two problems per wave (rows 0, 1) */
#define MHPC_VARIANT_BWS_ROWS1 3      /*   one problem per wave (row 0) */
#define MHPC_VARIANT_BWS_PAIRS2 4     /*   two problems per wave, two rows each in the
                                         whole-body phases (default up to 2048 problems) */
#define MHPC_VARIANT_RO 1             /* which: line-search rollouts */
#define MHPC_VARIANT_RO_PAIR 1        /*   two-wave pipeline, a lane pair per candidate */
#define MHPC_VARIANT_RO_PIPE_STAGED 2 /*   two-wave pipeline, LDS-staged operands */
#define MHPC_VARIANT_RO_PIPE 3        /*   two-wave pipeline, operands from HBM */
#define MHPC_VARIANT_RO_FUSED_STAGED 4 /*  one wave, LDS-staged operands */
#define MHPC_VARIANT_RO_FUSED 5       /*   one wave, operands from HBM */
#define MHPC_VARIANT_OVERLAP 2        /* which: partials beside the SRB half of the sweep */
#define MHPC_VARIANT_OVERLAP_ON 1     /*   two launches + second stream (default when both
                                         WB and SRB phases are present) */
#define MHPC_VARIANT_OVERLAP_OFF 2    /*   one sweep launch after the partials */
#define MHPC_VARIANT_SUBBATCH 3       /* which: sub-batches run concurrently; variant = their
                                         count 1..MHPC_MAX_SUBBATCH (contiguous blocks of the
                                         batch, one stream pair each, staggered by one launch
                                         so that one block's line search shares the chip with
                                         another block's sweep); 0 = automatic */
#define MHPC_MAX_SUBBATCH 4
#define MHPC_VARIANT_RO_STORE 4       /* which: line-search trials that store their knot
                                         records: the first `variant` (1..32) and the last;
                                         an accepted trial without records is rolled out again
                                         into its slot (same arithmetic, bit for bit);
                                         0 = the default (4) */
#define MHPC_VARIANT_SWEEP_BITS 5     /* which: arithmetic of the backward sweep: 64 (default,
                                         also in an fp32 handle, whose sweep reads float records
                                         and writes float gains but sums, factors and carries the
                                         value function in double) or, fp32 handles only, 32
                                         (the sweep in float, its 4x4 control block in double:
                                         faster, 10-70x larger typical error vs the fp64 oracle,
                                         DESIGN.md §5); 0 = default */
int mhpc_set_kernel_variant(mhpc_handle* h, int which, int variant);

/* ---- batched model evaluation on the device (kernel-level parity hooks) -----------
 * Replace the CasADi C ABI of SURVEY.md table 2b for whole batches of points.  All
 * arrays are host, row-major, n points.  Dense outputs: Ac/Px [n][14][14], Bc [n][14][4],
 * C [n][4][14], D [n][4][4]; SRB Ac [n][6][6], Bc [n][6][4]. */
int mhpc_eval_wb_dynamics(int device, int n, int mode, const double* x, const double* u,
                          double* xdot, double* y);
/* The line search's lane-pair evaluation of the same dynamics (mhpc_model_pair.h: even lane
 * front leg, odd lane back leg): xdot [n][2][14], y [n][2][4] hold what each lane of the pair
 * computed; both must equal mhpc_eval_wb_dynamics bit for bit. */
int mhpc_eval_wb_dynamics_pair(int device, int n, int mode, const double* x, const double* u,
                               double* xdot, double* y);
/* Touchdown constraint WB_FL1 (foot 0: front, used at the end of mode 2) / WB_FL2 (foot 1:
 * back, mode 4) and the foot Jacobian Jacob_F / Jacob_B, as the kernels evaluate them:
 * h [n][2] (the derivative routine's value, then the value-only routine's), hx [n][14],
 * hxx [n][14][14], J and Jd [n][2][7] (row-major). */
int mhpc_eval_wb_touchdown(int device, int n, int foot, const double* x, double* h, double* hx,
                           double* hxx, double* J, double* Jd);
/* The same two models in the fp32 instantiation (config C5): pair = 0 single lane (xdot
 * [n][14], y [n][4]), pair = 1 lane pair (xdot [n][2][14], y [n][2][4]); double host arrays,
 * inputs rounded to float. */
int mhpc_eval_wb_dynamics_f32(int device, int n, int mode, int pair, const double* x,
                              const double* u, double* xdot, double* y);
int mhpc_eval_wb_partials(int device, int n, int mode, const double* x, const double* u,
                          double* Ac, double* Bc, double* C, double* D);
int mhpc_eval_wb_impact(int device, int n, int foot, const double* x, double* xplus,
                        double* Px);
int mhpc_eval_srb(int device, int n, const double* x, const double* u, const double* foothold,
                  const double* contact, double* xdot, double* Ac, double* Bc);

#ifdef __cplusplus
}
#endif
#endif /* MHPC_CAPI_H */
