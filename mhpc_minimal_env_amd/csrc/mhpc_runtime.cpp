// Host runtime behind include/mhpc_capi.h: handle lifetime, HBM allocation, and the
// fixed kernel schedule of one batched solve (MultiPhaseDDP::solve restated as launches
// over a device-resident per-problem state machine).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <cmath>
#include <string>
#include <algorithm>
#include <map>
#include <numeric>
#include <vector>

#include "../../include/mhpc_capi.h"
#include "mhpc_solver.h"

namespace MHPC_NS {
hipError_t launch_init(const SolveParams&, const DevBufs&, hipStream_t);
hipError_t launch_reset_arrays(const SolveParams&, const DevBufs&, hipStream_t);
hipError_t launch_rollout(const SolveParams&, const DevBufs&, int, int, int, int, hipStream_t);
hipError_t launch_partials(const SolveParams&, const DevBufs&, hipStream_t, hipStream_t, hipEvent_t,
                           hipEvent_t);
hipError_t launch_bws(const SolveParams&, const DevBufs&, real, int, hipStream_t);
bool bws_split(const SolveParams&);
#ifdef MHPC_FP32
namespace fsweep {  // the float-arithmetic sweep (mhpc_bws.hip built with MHPC_BWS_F64=0)
hipError_t launch_bws(const SolveParams&, const DevBufs&, real, int, hipStream_t);
}
#endif
int ro_store_default();
int ro_store_auto(const SolveParams&);
hipError_t launch_cost(const SolveParams&, const DevBufs&, int, hipStream_t);
hipError_t launch_reset(const SolveParams&, const DevBufs&, hipStream_t);
hipError_t launch_store(const SolveParams&, const DevBufs&, real*, int, int, int, hipStream_t);
// N_TIMESTEPS_MAX (MHPCLocomotion.h): knots per phase buffer; record = x,u,y + K + du + G
constexpr int kPhaseBufKnots = 110;
constexpr int kStoreRec = KS + 56 + 4 + 14;
hipError_t launch_cost_grad(const SolveParams&, const DevBufs&, int, int, int, int, int, real*, real*,
                            hipStream_t);
hipError_t launch_eps_rollout(const SolveParams&, const DevBufs&, int, const real*, real*,
                              real*, hipStream_t);
hipError_t launch_al_end(const SolveParams&, const DevBufs&, int, hipStream_t);
hipError_t launch_export(const SolveParams&, const DevBufs&, hipStream_t);
hipError_t launch_reduce_counters(const SolveParams&, const DevBufs&, unsigned long long*,
                                  hipStream_t);
hipError_t launch_eval_wb_dyn(int, int, const real*, const real*, real*, real*, hipStream_t);
hipError_t launch_eval_wb_dyn_pair(int, int, const real*, const real*, real*, real*, hipStream_t);
#ifndef MHPC_FP32
hipError_t launch_eval_wb_par(int, int, const real*, const real*, real*, real*, real*,
                              real*, hipStream_t);
hipError_t launch_eval_wb_aux(int, int, const real*, real*, real*, real*, real*, real*, hipStream_t);
hipError_t launch_eval_wb_impact(int, int, const real*, real*, real*, hipStream_t);
hipError_t launch_eval_srb(int, const real*, const real*, const real*, const real*,
                           real*, real*, real*, hipStream_t);
#endif
}  // namespace MHPC_NS

extern thread_local std::string mhpc_g_err;  // mhpc_capi.cpp (mhpc_last_error)

#define API_NS MHPC_NS
#include "mhpc_api_decl.h"
#undef API_NS

namespace MHPC_NS {
namespace {
int fail(int code, const std::string& msg) {
  mhpc_g_err = msg;
  return code;
}

#define HIPCHK(expr)                                                                  \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess)                                                             \
      return fail(MHPC_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)
}  // namespace

enum { K_INIT = 0, K_FULL, K_LS, K_PAR, K_BWS, K_AL, K_BWS_SRB, NKERN };
static const char* kKernelNames[NKERN] = {"k_init", "k_cost(forward_sweep0)", "k_rollout(linesearch)",
                                          "k_partials", "k_bws", "k_al_end", "k_bws_srb"};

// Per-problem phase layout: the descriptor (gait point) and the phase-buffer rotation of the
// receding-horizon loop (MHPCLocomotion::update_problem rotates pidx_WB / pidx_FB by one per
// call, MHPCLocomotion.cpp:111-121: after r calls phase i uses buffer (i + r) mod n).
struct ProbLayout {
  mhpc_problem_desc desc;
  int rot_wb, rot_fb;
};
// Algorithmic bytes per problem of one layout
struct ByteModel {
  double roll_read = 0, roll_write = 0, roll_term = 0, par = 0, init = 0, cost = 0;
  double roll_flops = 0;  // one trial rollout (the line search's flop model)
};

struct Handle {
  mhpc_problem_desc desc;  // the descriptor of mhpc_create (precision, vel, height)
  mhpc_hsddp_option opt;
  int device = 0;
  SolveParams sp;
  DevBufs d;
  hipStream_t stream = nullptr;
  // second stream: the partials run there beside the SRB half of the backward sweep
  // (fork / join events order it against the main stream)
  hipStream_t stream2 = nullptr, stream3 = nullptr;  // stream3: the partials' second group
  hipEvent_t evfork = nullptr, evjoin = nullptr, evpfork = nullptr, evpjoin = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool x0_set = false, initialized = false, solved = false, x0_changed = false;
  // constraint parameters replaced after the last initialize / update_problem: their AL / ReB
  // initial values reach the problems' state only there, so a solve in between
  // would mix new limits with old initial values -- refused until then
  bool params_changed = false;
  float solve_ms = 0;
  unsigned long long* dcnt = nullptr;  // reduced counters per layout group [MAXL][NCNT]
  unsigned long long cnt[NCNT] = {};   // their sum over the groups
  unsigned long long gcnt[MAXL][NCNT] = {};
  // profiling: one event pair per launch of a solve, accumulated per kernel id
  bool profile = false;
  std::vector<hipEvent_t> evpool;
  std::vector<int> evkind;
  double kms[NKERN] = {}, kbytes[NKERN] = {}, kflops[NKERN] = {};
  int64_t klaunch[NKERN] = {};
  // per-problem layouts and the layout groups built from them (rebuild_groups): the layout
  // table (host / device), each problem's layout, the problems grouped by layout
  std::vector<ProbLayout> pl;
  std::vector<Layout> lays;
  std::vector<mhpc_problem_desc> ldesc;  // descriptor of each layout
  std::vector<int> lid, gidx;
  Layout* dlay = nullptr;
  int *dgidx = nullptr, *dlid = nullptr;
  // algorithmic byte model per problem of each layout
  std::vector<ByteModel> bym;
  // receding horizon (MHPCLocomotion::update_problem): each problem's current mode, the
  // buffer store [B][spmax][nbk] (allocated at the first update), knot capacity of the
  // packed arrays, and whether the next solve's first forward_sweep(0) must be a real
  // rollout (rotated nominal, new x0)
  std::vector<int> cmode;
  real* store = nullptr;
  int nbk = 0, nk_cap = 0, spmax = 0;
  bool need_full = false;
  bool store_valid = false;  // store zeroed since the last initialize (memory_reset)
  // sub-batches (MHPC_VARIANT_SUBBATCH): the solve schedule runs once per contiguous block of
  // problems, each block on its own stream pair; created on first use
  int nsub_req = 0;
  int ro_store_req = 0;  // MHPC_VARIANT_RO_STORE (0: by the batch's line-search shape)
  int sweep_bits = 0;    // MHPC_VARIANT_SWEEP_BITS (0 = 64: the sweep computes in double)
  struct SubStreams {
    hipStream_t s1 = nullptr, s2 = nullptr, s3 = nullptr;  // s3: the partials' second group
    hipEvent_t fork = nullptr, join = nullptr, gate = nullptr, done = nullptr, pfork = nullptr,
               pjoin = nullptr;
  };
  std::vector<SubStreams> subs;
  hipEvent_t evstart = nullptr;
};

// Phase layout of a descriptor: modes, knot counts and offsets, partials work items, and the
// phase buffers after rot_wb / rot_fb rotations (MHPCLocomotion::update_problem).
static void build_layout(Layout& L, const mhpc_problem_desc& desc, int rot_wb, int rot_fb) {
  memset(&L, 0, sizeof L);
  L.P = desc.n_wb + desc.n_fb;
  L.n_wb = desc.n_wb;
  int ko = 0, items = 0, items_v = 0;
  for (int p = 0; p < L.P; ++p) {
    const bool wb = p < desc.n_wb;
    L.mode[p] = desc.mode_seq[p];
    L.N[p] = desc.N[p];
    L.ko[p] = ko;
    L.xs[p] = wb ? 14 : 6;
    L.dt[p] = wb ? desc.dt_wb : desc.dt_fb;
    L.buf[p] = wb ? (p + rot_wb) % desc.n_wb : desc.n_wb + (p - desc.n_wb + rot_fb) % desc.n_fb;
    ko += desc.N[p];
    L.par_knot_off[p] = items;
    L.par_imp_off[p] = items_v;
    if (wb) {
      items += desc.N[p] - 1;
      items_v += (L.mode[p] == 2 || L.mode[p] == 4) ? 14 : 0;
    }
  }
  for (int p = L.P; p <= MAXP; ++p) {
    L.par_knot_off[p] = items;
    L.par_imp_off[p] = items_v;
  }
  L.par_knots = items;
  L.par_imp = items_v;
  L.NK = ko;
}

// Algorithmic HBM bytes (fp64) of one problem for each kernel's unit of work.
constexpr double kB = sizeof(real);  // bytes per element of the solve's arithmetic type

// Line-search flop model per trial knot (SURVEY.md 8d secondary roofline): the reference's
// dynamics in CasADi's generated-code assignment counts (Dyn_BS / Dyn_FS 2301,
// Dyn_FL 1441, FBDynamics 44 -- scalar operations incl. loads, so an upper estimate), plus the
// feedback u = u_nom + eps du + K (x - x_nom) and the Euler step (WB: 14 + 4 * 28 + 8 + 28;
// SRB: 6 + 4 * 12 + 8 + 12).  The running costs (the second wave) are not counted.
static double ro_knot_flops(int mode, bool wb) {
  if (!wb) return 44 + 74;
  return (mode == 1 || mode == 3 ? 2301.0 : 1441.0) + 162;
}

static ByteModel byte_model(const Layout& L) {
  ByteModel m;
  double rr = 14 * 8, rw = 0, rt = 0, pb = 0, ib = L.NK * kB, cb = 0;
  for (int p = 0; p < L.P; ++p) {
    const bool wb = p < L.n_wb;
    const int n = wb ? 14 : 6, N = L.N[p];
    // nominal x,u (n+4) + K (4n) + du (4) read once per problem (the candidates of a
    // problem share them)
    rr += (N - 1) * kB * ((n + 4) + 4 * n + 4);
    // a storing candidate writes x,u,y of every knot, every candidate x at the last knot
    rw += (N - 1) * kB * (n + 8);
    rt += n * kB;
    m.roll_flops += (N - 1) * ro_knot_flops(L.mode[p], wb);
    // k_cost: nominal x,u(,y) of every knot + refpos
    cb += (N - 1) * kB * (n + 4 + (wb ? 4 : 0) + 1) + kB * (n + 1);
    // k_init: x,u,y written for every knot (WB and SRB)
    if (!wb) ib += N * kB * 14;
    if (wb) {
      const bool imp = L.mode[p] == 2 || L.mode[p] == 4;
      // x,u read; the record written without its four zero columns (written once at create)
      pb += (N - 1) * kB * (18 + PS - 4 * 9) + (imp ? kB * (14 + 196) : 0.0);
      ib += N * kB * 22;
    }
  }
  m.roll_read = rr;
  m.roll_write = rw;
  m.roll_term = rt;
  m.par = pb;
  m.init = ib;
  m.cost = cb;
  return m;
}
// backward sweep: per WB knot partials record + x,u,y + refpos read, K,du,G written;
// per SRB knot x,u + refpos read, K,du,G written; Px read per impact-aware step
static constexpr double kBwsWbKnot = kB * (PS + 22 + 1 + 56 + 4 + 14);
static constexpr double kBwsFbKnot = kB * (10 + 1 + 24 + 4 + 6);
static constexpr double kBwsPx = kB * 196;
// Algorithmic FP64 flops of the backward sweep in the reference's dense formulation
// (compute_Qfunction 20.2k + valuefunction_update 4.3k per WB knot,
// ~3k per SRB knot; impact_aware_step Px' G, Px' H Px: 2 (2 * 14^3) + 2 * 14^2).  The
// kernel skips the structural zeros, so this is the dense-equivalent rate, an upper bound
// on the flops it executes.
static constexpr double kFlopWbKnot = 24.5e3, kFlopFbKnot = 3.0e3,
                        kFlopPx = 2.0 * (2.0 * 14 * 14 * 14) + 2.0 * 14 * 14;

const char* api_kernel_name(int k) {
  return (k >= 0 && k < NKERN) ? kKernelNames[k] : "";
}


static int validate(const mhpc_problem_desc* d) {
  if (!d) return fail(MHPC_ERR_INVALID, "null descriptor");
  const int P = d->n_wb + d->n_fb;
  if (d->n_wb < 0 || d->n_fb < 0 || P < 1 || P > MHPC_MAX_PHASES)
    return fail(MHPC_ERR_INVALID, "phase count out of range");
  if (d->precision != 64 && d->precision != 32) return fail(MHPC_ERR_INVALID, "precision must be 64 or 32");
  int NK = 0;
  for (int p = 0; p < P; ++p) {
    if (d->mode_seq[p] < 1 || d->mode_seq[p] > 4) return fail(MHPC_ERR_INVALID, "mode out of range");
    if (d->N[p] < 2) return fail(MHPC_ERR_INVALID, "each phase needs N >= 2");
    NK += d->N[p];
  }
  if (NK > MHPC_MAX_KNOTS) return fail(MHPC_ERR_INVALID, "too many knots");
  if (!(d->dt_wb > 0) || !(d->dt_fb > 0)) return fail(MHPC_ERR_INVALID, "dt must be positive");
  return MHPC_OK;
}


static void free_bufs(Handle* h) {
  DevBufs& d = h->d;
  void* ptrs[] = {d.traj, d.refpos, d.K, d.du, d.G, d.par, d.px, d.x0, d.st, d.out, d.carry,
                  h->dlay, h->dgidx, h->dlid};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  memset(&d, 0, sizeof d);
  h->dlay = nullptr;
  h->dgidx = h->dlid = nullptr;
}

// A descriptor normalised for comparison (entries past its phases and reserved fields zero)
static mhpc_problem_desc norm_desc(const mhpc_problem_desc& in) {
  mhpc_problem_desc d;
  memset(&d, 0, sizeof d);
  d.n_wb = in.n_wb;
  d.n_fb = in.n_fb;
  for (int p = 0; p < in.n_wb + in.n_fb; ++p) {
    d.mode_seq[p] = in.mode_seq[p];
    d.N[p] = in.N[p];
  }
  d.dt_wb = in.dt_wb;
  d.dt_fb = in.dt_fb;
  d.vel_cmd = in.vel_cmd;
  d.height_cmd = in.height_cmd;
  d.precision = in.precision;
  return d;
}

// The packed per-knot arrays for a knot stride of NK (grown, never shrunk: their content is
// rebuilt by initialize / update_problem).  The partials records' zero columns (x, z, xdot,
// zdot) are written by no kernel: they are zeroed here whenever the stride changes, since the
// column blocks are stride-major (par_col) and a new stride moves them onto words the old
// stride used for other columns.  New arrays are allocated before the old ones are freed, so
// a failed allocation leaves the handle's arrays and stride as they were.
static int ensure_knot_arrays(Handle* h, int NK) {
  DevBufs& d = h->d;
  const size_t B = h->sp.B, nk = NK;
  const bool grow = NK > h->nk_cap;
  if (!grow && NK == h->sp.NK) return MHPC_OK;
  HIPCHK(hipStreamSynchronize(h->stream));
  HIPCHK(hipStreamSynchronize(h->stream2));
  HIPCHK(hipStreamSynchronize(h->stream3));
  for (const Handle::SubStreams& s : h->subs) {
    if (s.s1) HIPCHK(hipStreamSynchronize(s.s1));
    if (s.s2) HIPCHK(hipStreamSynchronize(s.s2));
    if (s.s3) HIPCHK(hipStreamSynchronize(s.s3));
  }
  if (grow) {
    real** arr[] = {&d.traj, &d.refpos, &d.K, &d.du, &d.G, &d.par, &d.out};
    const size_t per[] = {(size_t)h->sp.nslot * KS, 1, 56, 4, 14, PS, KS};
    real* fresh[7] = {};
    for (int i = 0; i < 7; ++i) {
      const hipError_t e = hipMalloc((void**)&fresh[i], B * nk * per[i] * sizeof(real));
      if (e != hipSuccess) {
        for (int j = 0; j < i; ++j) (void)hipFree(fresh[j]);
        return fail(MHPC_ERR_DEVICE, std::string("knot array allocation failed: ") + hipGetErrorString(e));
      }
    }
    for (int i = 0; i < 7; ++i) {
      if (*arr[i]) (void)hipFree(*arr[i]);
      *arr[i] = fresh[i];
    }
    h->nk_cap = NK;
    HIPCHK(hipMemsetAsync(d.traj, 0, B * h->sp.nslot * nk * KS * sizeof(real), h->stream));
  }
  HIPCHK(hipMemsetAsync(d.par, 0, B * nk * PS * sizeof(real), h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return MHPC_OK;
}

// Layout groups from the per-problem layouts: the distinct (descriptor, buffer rotation)
// pairs, longest layout first (its blocks head every launch: the long blocks start first in a
// mixed batch), the problems of each group in batch order.  Uploads the layout table and the
// grouped order, sets the launch fields of sp, grows the packed arrays if a layout needs it.
static int rebuild_groups(Handle* h) {
  SolveParams& sp = h->sp;
  const int B = sp.B;
  std::map<std::string, int> seen;
  std::vector<ProbLayout> uniq;
  std::vector<int> first_lid(B);
  for (int b = 0; b < B; ++b) {
    ProbLayout k;
    memset(&k, 0, sizeof k);
    k.desc = norm_desc(h->pl[b].desc);
    k.rot_wb = k.desc.n_wb > 0 ? h->pl[b].rot_wb % k.desc.n_wb : 0;
    k.rot_fb = k.desc.n_fb > 0 ? h->pl[b].rot_fb % k.desc.n_fb : 0;
    const std::string key((const char*)&k, sizeof k);
    auto it = seen.find(key);
    if (it == seen.end()) {
      if ((int)uniq.size() == MAXL) return fail(MHPC_ERR_INVALID, "more than MHPC_MAX_LAYOUTS distinct layouts");
      it = seen.emplace(key, (int)uniq.size()).first;
      uniq.push_back(k);
    }
    first_lid[b] = it->second;
  }
  const int L = (int)uniq.size();
  std::vector<Layout> lay(L);
  for (int l = 0; l < L; ++l) build_layout(lay[l], uniq[l].desc, uniq[l].rot_wb, uniq[l].rot_fb);
  std::vector<int> order(L), rank(L);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int a, int c) { return lay[a].NK > lay[c].NK; });
  for (int g = 0; g < L; ++g) rank[order[g]] = g;
  h->lays.resize(L);
  h->ldesc.resize(L);
  h->bym.resize(L);
  int NK = 0, pmax = 0;
  sp.split_ok = 0;
  sp.stage_fits = 1;
  for (int g = 0; g < L; ++g) {
    const Layout& Lg = lay[order[g]];
    h->lays[g] = Lg;
    h->ldesc[g] = uniq[order[g]].desc;
    h->bym[g] = byte_model(Lg);
    NK = std::max(NK, Lg.NK);
    pmax = std::max(pmax, Lg.P);
    if (Lg.n_wb > 0 && Lg.P > Lg.n_wb) sp.split_ok = 1;
    for (int p = 0; p < Lg.P; ++p)
      if (Lg.N[p] > ST_RMAX) sp.stage_fits = 0;
    sp.gpk[g] = Lg.par_knots;
    sp.gpi[g] = Lg.par_imp;
  }
  h->lid.resize(B);
  std::vector<int> cnt(L + 1, 0);
  for (int b = 0; b < B; ++b) {
    h->lid[b] = rank[first_lid[b]];
    ++cnt[h->lid[b] + 1];
  }
  sp.ngrp = L;
  for (int g = 0; g < L; ++g) cnt[g + 1] += cnt[g];
  for (int g = 0; g <= L; ++g) sp.go[g] = cnt[g];
  h->gidx.resize(B);
  sp.ident = 1;
  for (int b = 0; b < B; ++b) {
    const int pos = cnt[h->lid[b]]++;
    h->gidx[pos] = b;
    if (pos != b) sp.ident = 0;
  }
  sp.pmax = pmax;
  int rc = ensure_knot_arrays(h, NK);
  if (rc) return rc;
  sp.NK = NK;
  h->d.lay = h->dlay;
  h->d.gidx = h->dgidx;
  h->d.lid = h->dlid;
  HIPCHK(hipMemcpyAsync(h->dlay, h->lays.data(), L * sizeof(Layout), hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->dgidx, h->gidx.data(), B * sizeof(int), hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->dlid, h->lid.data(), B * sizeof(int), hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return MHPC_OK;
}

// Host (double) parameter structs <-> the kernels' parameter block (real).
static void put_weights(CostParams& cw, const mhpc_cost_weights& w) {
  for (int m = 0; m < 4; ++m) {
    for (int i = 0; i < 14; ++i) {
      cw.wQ[m][i] = (real)w.wb_Q[m][i];
      cw.wQf[m][i] = (real)w.wb_Qf[m][i];
    }
    for (int i = 0; i < 4; ++i) {
      cw.wR[m][i] = (real)w.wb_R[m][i];
      cw.wS[m][i] = (real)w.wb_S[m][i];
      cw.fR[m][i] = (real)w.fb_R[m][i];
    }
    for (int i = 0; i < 6; ++i) {
      cw.fQ[m][i] = (real)w.fb_Q[m][i];
      cw.fQf[m][i] = (real)w.fb_Qf[m][i];
    }
  }
}
static void get_weights(const CostParams& cw, mhpc_cost_weights& w) {
  for (int m = 0; m < 4; ++m) {
    for (int i = 0; i < 14; ++i) {
      w.wb_Q[m][i] = cw.wQ[m][i];
      w.wb_Qf[m][i] = cw.wQf[m][i];
    }
    for (int i = 0; i < 4; ++i) {
      w.wb_R[m][i] = cw.wR[m][i];
      w.wb_S[m][i] = cw.wS[m][i];
      w.fb_R[m][i] = cw.fR[m][i];
    }
    for (int i = 0; i < 6; ++i) {
      w.fb_Q[m][i] = cw.fQ[m][i];
      w.fb_Qf[m][i] = cw.fQf[m][i];
    }
  }
}
static void put_constraints(CostParams& cw, const mhpc_constraint_params& c) {
  cw.tq_lim = (real)c.torque_limit;
  cw.mu = (real)c.friction_coeff;
  for (int m = 0; m < 4; ++m) {
    cw.sigma0[m] = (real)c.sigma[m];
    cw.delta0[m] = (real)c.delta[m];
    cw.delta_min[m] = (real)c.delta_min[m];
    cw.eps_tq0[m] = (real)c.eps_torque[m];
    cw.eps_grf0[m] = (real)c.eps_grf[m];
  }
}
static void get_constraints(const CostParams& cw, mhpc_constraint_params& c) {
  c.torque_limit = cw.tq_lim;
  c.friction_coeff = cw.mu;
  for (int m = 0; m < 4; ++m) {
    c.sigma[m] = cw.sigma0[m];
    c.delta[m] = cw.delta0[m];
    c.delta_min[m] = cw.delta_min[m];
    c.eps_torque[m] = cw.eps_tq0[m];
    c.eps_grf[m] = cw.eps_grf0[m];
  }
}

int api_set_cost_weights(Handle* h, const mhpc_cost_weights* w) {
  if (!h || !w) return fail(MHPC_ERR_INVALID, "null argument");
  const double* v = &w->wb_Q[0][0];
  for (size_t i = 0; i < sizeof(mhpc_cost_weights) / sizeof(double); ++i)
    if (!std::isfinite(v[i]) || v[i] < 0) return fail(MHPC_ERR_INVALID, "cost weights must be finite and >= 0");
  put_weights(h->sp.cw, *w);
  return MHPC_OK;
}
int api_get_cost_weights(Handle* h, mhpc_cost_weights* w) {
  if (!h || !w) return fail(MHPC_ERR_INVALID, "null argument");
  get_weights(h->sp.cw, *w);
  return MHPC_OK;
}
int api_set_constraint_params(Handle* h, const mhpc_constraint_params* c) {
  if (!h || !c) return fail(MHPC_ERR_INVALID, "null argument");
  const double* v = &c->torque_limit;
  for (size_t i = 0; i < sizeof(mhpc_constraint_params) / sizeof(double); ++i)
    if (!std::isfinite(v[i])) return fail(MHPC_ERR_INVALID, "constraint parameters must be finite");
  if (!(c->torque_limit > 0)) return fail(MHPC_ERR_INVALID, "torque_limit must be > 0");
  if (!(c->friction_coeff >= 0))
    return fail(MHPC_ERR_INVALID, "friction_coeff must be >= 0 (a negative one inverts the GRF cone)");
  for (int m = 0; m < 4; ++m) {
    if (!(c->delta[m] > 0) || !(c->delta_min[m] > 0))
      return fail(MHPC_ERR_INVALID, "delta and delta_min must be > 0");
    if (c->delta_min[m] > c->delta[m])
      return fail(MHPC_ERR_INVALID, "delta_min must not exceed delta (the AL update only shrinks delta)");
    if (c->sigma[m] < 0 || c->eps_torque[m] < 0 || c->eps_grf[m] < 0)
      return fail(MHPC_ERR_INVALID, "sigma and the ReB weights must be >= 0");
  }
  put_constraints(h->sp.cw, *c);
  if (h->initialized) h->params_changed = true;
  return MHPC_OK;
}
int api_get_constraint_params(Handle* h, mhpc_constraint_params* c) {
  if (!h || !c) return fail(MHPC_ERR_INVALID, "null argument");
  get_constraints(h->sp.cw, *c);
  return MHPC_OK;
}

int api_create(const mhpc_problem_desc* desc, const mhpc_hsddp_option* opt, int batch,
                           int device, Handle** out) {
  if (!out || !opt) return fail(MHPC_ERR_INVALID, "null argument");
  *out = nullptr;
  int rc = validate(desc);
  if (rc) return rc;
  if (batch < 1) return fail(MHPC_ERR_INVALID, "batch must be >= 1");
  if (!(opt->alpha > 0 && opt->alpha < 1)) return fail(MHPC_ERR_INVALID, "alpha must be in (0,1)");
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(MHPC_ERR_INVALID, "no such device");
  HIPCHK(hipSetDevice(device));

  Handle* h = new Handle();
  h->desc = norm_desc(*desc);
  h->opt = *opt;
  h->device = device;
  SolveParams& sp = h->sp;
  memset(&sp, 0, sizeof sp);
  sp.B = batch;
  // launch shapes follow this handle's device (one process may hold handles on several)
  if (hipDeviceGetAttribute(&sp.ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
      sp.ncu < 1)
    sp.ncu = 256;
  sp.vel = desc->vel_cmd;
  sp.height = desc->height_cmd;
  // line-search grid exactly as MultiPhaseDDP::forward_iteration generates it (:130-151)
  int nc = 0;
  for (double eps = 1; eps > pow(0.1, 10); eps *= opt->alpha) {
    if (nc == MAXC) {
      delete h;
      return fail(MHPC_ERR_INVALID, "line search needs more than 32 trials (alpha too large)");
    }
    sp.eps[nc++] = eps;
  }
  sp.n_cand = nc;
  sp.ro_store = ro_store_default();
  sp.nslot = nc + 1;
  sp.gamma = opt->gamma;
  sp.DDP_thresh = opt->DDP_thresh;
  sp.AL_thresh = opt->AL_thresh;
  sp.update_penalty = opt->update_penalty;
  sp.update_relax = opt->update_relax;
  sp.update_regularization = opt->update_regularization;
  sp.update_ReB = opt->update_ReB;
  sp.eps9 = pow(0.1, 9);
  sp.AL_active = opt->AL_active ? 1 : 0;
  sp.ReB_active = opt->ReB_active ? 1 : 0;
  {  // the reference's weights and constraint parameters until mhpc_set_* replaces them
    mhpc_cost_weights w;
    mhpc_constraint_params c;
    mhpc_default_cost_weights(&w);
    mhpc_default_constraint_params(&c);
    put_weights(sp.cw, w);
    put_constraints(sp.cw, c);
  }
  h->pl.assign(batch, ProbLayout{h->desc, 0, 0});
  h->cmode.assign(batch, desc->mode_seq[0]);

  DevBufs& d = h->d;
  memset(&d, 0, sizeof d);
  const size_t B = batch;
  hipError_t e = hipSuccess;
  auto alloc = [&](void** p, size_t bytes) {
    if (e == hipSuccess) e = hipMalloc(p, bytes);
  };
  alloc((void**)&d.px, B * MAXP * 196 * sizeof(real));
  alloc((void**)&d.x0, B * 14 * sizeof(real));
  alloc((void**)&d.st, B * sizeof(ProbState));
  alloc((void**)&d.carry, B * sizeof(BwsCarry));
  alloc((void**)&h->dcnt, MAXL * NCNT * sizeof(unsigned long long));
  alloc((void**)&h->dlay, MAXL * sizeof(Layout));
  alloc((void**)&h->dgidx, B * sizeof(int));
  alloc((void**)&h->dlid, B * sizeof(int));
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->stream2, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&h->evfork, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&h->evjoin, hipEventDisableTiming);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->stream3, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&h->evpfork, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&h->evpjoin, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreate(&h->ev0);
  if (e == hipSuccess) e = hipEventCreate(&h->ev1);
  // zero x0 on the handle's own (non-blocking) stream: a null-stream memset would not be
  // ordered before mhpc_set_x0's copy on this stream
  if (e == hipSuccess) e = hipMemsetAsync(d.x0, 0, B * 14 * sizeof(real), h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  int rc2 = e == hipSuccess ? MHPC_OK : fail(MHPC_ERR_DEVICE, std::string("allocation failed: ") + hipGetErrorString(e));
  if (!rc2) rc2 = rebuild_groups(h);  // one layout group; allocates the packed arrays
  if (rc2) {
    api_destroy(h);
    return rc2;
  }
  *out = h;
  return MHPC_OK;
}

static int x0_row(const Handle* h) {
  for (const Layout& L : h->lays)
    if (L.n_wb > 0) return 14;
  return 6;
}

int api_set_x0(Handle* h, const double* x0) {
  if (!h || !x0) return fail(MHPC_ERR_INVALID, "null argument");
  HIPCHK(hipSetDevice(h->device));
  // rows of 14 when any layout starts with a whole-body phase (an SRB-only problem reads the
  // first 6 entries of its row), else 6
  const int n0 = x0_row(h);
  std::vector<real> pad((size_t)h->sp.B * 14, real(0));
  for (int b = 0; b < h->sp.B; ++b) {
    const int nb = h->lays[h->lid[b]].n_wb > 0 ? 14 : 6;
    for (int i = 0; i < nb; ++i) pad[(size_t)b * 14 + i] = (real)x0[(size_t)b * n0 + i];
  }
  HIPCHK(hipMemcpyAsync(h->d.x0, pad.data(), pad.size() * sizeof(real), hipMemcpyHostToDevice,
                        h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  h->x0_set = true;
  h->x0_changed = true;  // references follow x0 only through initialize / update_problem
  return MHPC_OK;
}

static int mark(Handle* h, int kind, hipStream_t s) {
  if (!h->profile) return MHPC_OK;
  hipEvent_t e;
  HIPCHK(hipEventCreate(&e));
  HIPCHK(hipEventRecord(e, s));
  h->evpool.push_back(e);
  h->evkind.push_back(kind);
  return MHPC_OK;
}
// one launch on stream s, bracketed by profiling events on the same stream
#define LAUNCH_ON(h, kind, s, expr)    \
  do {                                 \
    int rc_ = mark(h, kind, s);        \
    if (rc_) return rc_;               \
    HIPCHK(expr);                      \
    rc_ = mark(h, -1, s);              \
    if (rc_) return rc_;               \
  } while (0)
#define LAUNCH(h, kind, expr) LAUNCH_ON(h, kind, h->stream, expr)

static int collect_profile(Handle* h) {
  for (size_t i = 0; i + 1 < h->evpool.size(); i += 2) {
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, h->evpool[i], h->evpool[i + 1]));
    h->kms[h->evkind[i]] += ms;
    h->klaunch[h->evkind[i]] += 1;
  }
  for (hipEvent_t e : h->evpool) (void)hipEventDestroy(e);
  h->evpool.clear();
  h->evkind.clear();
  return MHPC_OK;
}

// Device -> host copy ordered on the handle's stream.
static int d2h(Handle* h, void* dst, const void* src, size_t bytes) {
  HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return MHPC_OK;
}
#define D2H(dst, src, bytes)                \
  do {                                      \
    int rc_ = d2h(h, (dst), (src), (bytes)); \
    if (rc_) return rc_;                    \
  } while (0)

// initialization(): memory_reset + build_problem (refs) + warmstart, all on the device.
static int initialize_async(Handle* h) {
  // build_problem binds phase p to buffer p and starts the gait at each problem's first mode
  bool rotated = false;
  for (int b = 0; b < h->sp.B; ++b) {
    ProbLayout& q = h->pl[b];
    rotated = rotated || q.rot_wb != 0 || q.rot_fb != 0;
    q.rot_wb = q.rot_fb = 0;
    h->cmode[b] = q.desc.mode_seq[0];
  }
  if (rotated) {
    const int rc = rebuild_groups(h);
    if (rc) return rc;
  }
  const SolveParams& sp = h->sp;
  DevBufs& d = h->d;
  // memory_reset (K / du / G, trajectory tails) on the second stream beside k_init, which
  // touches none of it; the first solve op waits for both
  HIPCHK(hipEventRecord(h->evfork, h->stream));
  HIPCHK(hipStreamWaitEvent(h->stream2, h->evfork, 0));
  HIPCHK(launch_reset_arrays(sp, d, h->stream2));
  HIPCHK(hipEventRecord(h->evjoin, h->stream2));
  LAUNCH(h, K_INIT, launch_init(sp, d, h->stream));
  HIPCHK(hipStreamWaitEvent(h->stream, h->evjoin, 0));
  for (int g = 0; g < sp.ngrp; ++g) h->kbytes[K_INIT] += h->bym[g].init * (sp.go[g + 1] - sp.go[g]);
  // the buffer store is zeroed lazily (first update_problem), so a plain initialize + solve
  // pays nothing for it
  h->store_valid = false;
  h->need_full = false;
  return MHPC_OK;
}

int api_initialize(Handle* h) {
  if (!h) return fail(MHPC_ERR_INVALID, "null handle");
  if (!h->x0_set) return fail(MHPC_ERR_STATE, "mhpc_set_x0 must precede mhpc_initialize");
  HIPCHK(hipSetDevice(h->device));
  int rc = initialize_async(h);
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(h->stream));
  rc = collect_profile(h);
  if (rc) return rc;
  h->initialized = true;
  h->x0_changed = false;
  h->params_changed = false;
  h->solved = false;
  return MHPC_OK;
}

// MultiPhaseDDP::solve (MultiPhaseDDP.cpp:154-289) as a fixed launch schedule; every kernel
// skips the problems whose device state machine has left the corresponding loop.
// With bws_split the partials of an iteration run on the second stream beside the SRB half
// of the backward sweep (which reads no partials record); the WB half waits for them.
//
// Sub-batches (MHPC_VARIANT_SUBBATCH): the same schedule runs once per contiguous block of
// problems, each block on its own stream pair.  Problems are independent and every array is
// problem-major, so a block is a pointer offset and its problems compute exactly what they
// compute in one launch over the whole batch (every launch shape is bitwise the same
// arithmetic, tests/test_gpu_variants.py).  Block s+1 starts one launch behind block s:
// the line search (two thirds of the SIMDs busy at batch 1024, one wave per SIMD) then
// shares the chip with the other block's sweep / partials instead of leaving SIMDs idle.
enum { OP_COST, OP_FULL, OP_PAR, OP_BWS, OP_LS, OP_AL };
struct SolveOp {
  int kind, al, ddp, max_ddp;
};
struct SolveBlock {
  SolveParams sp;
  DevBufs d;
  hipStream_t s1, s2, s3;
  hipEvent_t fork, join, pfork, pjoin;
};

// Problems [b0, b0 + sp.B) of the handle's arrays as the kernels index them (b * per-problem
// stride, with sp.NK the knot stride of the packed arrays): for the layout-free export kernel.
static DevBufs block_bufs(const DevBufs& d, const SolveParams& sp, size_t b0) {
  DevBufs o = d;
  const size_t NK = sp.NK;
  o.traj += b0 * sp.nslot * NK * KS;
  o.refpos += b0 * NK;
  o.K += b0 * NK * 56;
  o.du += b0 * NK * 4;
  o.G += b0 * NK * 14;
  o.par += b0 * NK * PS;
  o.px += b0 * MAXP * 196;
  o.x0 += b0 * 14;
  o.st += b0;
  o.out += b0 * NK * KS;
  o.carry += b0;
  return o;
}

static std::vector<SolveOp> solve_ops(const Handle* h) {
  const mhpc_hsddp_option& o = h->opt;
  std::vector<SolveOp> ops;
  int n_al = 0;
  for (int al = 1; al <= o.max_AL_iter; ++al) n_al = al;
  int max_ddp = 0;
  for (int ddp = 1; ddp <= o.max_DDP_iter; ++ddp) max_ddp = ddp;
  for (int al = 1; al <= n_al; ++al) {
    // forward_sweep(0); a real rollout for the rotated nominal of update_problem
    ops.push_back({al == 1 && h->need_full ? OP_FULL : OP_COST, al, 0, 0});
    ops.push_back({OP_PAR, al, 0, 0});
    for (int ddp = 1; ddp <= max_ddp; ++ddp) {
      ops.push_back({OP_BWS, al, ddp, max_ddp});
      ops.push_back({OP_LS, al, ddp, max_ddp});  // forward_iteration
      if (ddp < max_ddp) ops.push_back({OP_PAR, al, ddp, max_ddp});
    }
    ops.push_back({OP_AL, al == n_al ? 1 : 0, 0, 0});
  }
  if (n_al == 0) ops.push_back({OP_AL, 1, 0, 0});
  return ops;
}

// With bws_split the partials run on the block's second stream beside the SRB half of the
// backward sweep (which reads no partials record); the WB half waits for them.
static int issue_op(Handle* h, const SolveBlock& k, const SolveOp& op) {
  const SolveParams& sp = k.sp;
  const DevBufs& d = k.d;
  const real ureg = h->opt.update_regularization;
  const bool split = bws_split(sp);
#ifdef MHPC_FP32
  auto launch_bws = h->sweep_bits == 32 ? fsweep::launch_bws : MHPC_NS::launch_bws;
#endif
  switch (op.kind) {
    case OP_FULL:
      LAUNCH_ON(h, K_FULL, k.s1, launch_rollout(sp, d, op.al, 0, 0, 1, k.s1));
      break;
    case OP_COST:
      LAUNCH_ON(h, K_FULL, k.s1, launch_cost(sp, d, op.al, k.s1));
      break;
    case OP_PAR:
      if (!split) {
        LAUNCH_ON(h, K_PAR, k.s1, launch_partials(sp, d, k.s1, k.s3, k.pfork, k.pjoin));
        break;
      }
      HIPCHK(hipEventRecord(k.fork, k.s1));
      HIPCHK(hipStreamWaitEvent(k.s2, k.fork, 0));
      LAUNCH_ON(h, K_PAR, k.s2, launch_partials(sp, d, k.s2, k.s3, k.pfork, k.pjoin));
      HIPCHK(hipEventRecord(k.join, k.s2));
      break;
    case OP_BWS:
      if (!split) {
        LAUNCH_ON(h, K_BWS, k.s1, launch_bws(sp, d, ureg, 0, k.s1));
        break;
      }
      LAUNCH_ON(h, K_BWS_SRB, k.s1, launch_bws(sp, d, ureg, 1, k.s1));
      HIPCHK(hipStreamWaitEvent(k.s1, k.join, 0));
      LAUNCH_ON(h, K_BWS, k.s1, launch_bws(sp, d, ureg, 2, k.s1));
      break;
    case OP_LS:
      LAUNCH_ON(h, K_LS, k.s1, launch_rollout(sp, d, op.al, op.ddp, op.max_ddp, 0, k.s1));
      break;
    default:
      LAUNCH_ON(h, K_AL, k.s1, launch_al_end(sp, d, op.al, k.s1));
  }
  return MHPC_OK;
}

static int sub_batches(const Handle* h) {
  int n = h->nsub_req;
  if (n == 0) n = 1;  // automatic: one block (DESIGN.md §3 has the measured A/B)
  return std::min(n, h->sp.B);
}

static int ensure_sub_streams(Handle* h, int n) {
  if (!h->evstart) HIPCHK(hipEventCreateWithFlags(&h->evstart, hipEventDisableTiming));
  while ((int)h->subs.size() < n) {
    h->subs.emplace_back();
    Handle::SubStreams& s = h->subs.back();
    HIPCHK(hipStreamCreateWithFlags(&s.s1, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&s.s2, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&s.s3, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&s.pfork, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&s.pjoin, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&s.fork, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&s.join, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&s.gate, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
  }
  return MHPC_OK;
}

static int solve_async(Handle* h) {
  // stored line-search trials for this batch's launch shape (unless set by the caller)
  if (!h->ro_store_req) h->sp.ro_store = ro_store_auto(h->sp);
  const std::vector<SolveOp> ops = solve_ops(h);
  const int nops = (int)ops.size();
  const int nsub = sub_batches(h);
  int rc;
  if (nsub <= 1) {
    const SolveBlock k{h->sp,       h->d,      h->stream,  h->stream2, h->stream3,
                       h->evfork,   h->evjoin, h->evpfork, h->evpjoin};
    for (const SolveOp& op : ops)
      if ((rc = issue_op(h, k, op))) {
        // an issue failure may leave launches queued on the second / third stream (the
        // partials fork onto stream3 and join back only at their end): drain both, so no later
        // work on the handle runs unordered with them
        (void)hipStreamSynchronize(h->stream3);
        (void)hipStreamSynchronize(h->stream2);
        (void)hipStreamWaitEvent(h->stream, h->evjoin, 0);
        return rc;
      }
    // a schedule whose last partials have no sweep after them (max_DDP_iter = 0) still
    // joins the second stream back before the solve counts as done
    HIPCHK(hipStreamWaitEvent(h->stream, h->evjoin, 0));
  } else {
    if ((rc = ensure_sub_streams(h, nsub))) return rc;
    HIPCHK(hipEventRecord(h->evstart, h->stream));
    std::vector<SolveBlock> blk(nsub);
    // even partition: every block non-empty (sub_batches() <= B), sizes differ by <= 1
    const int B = h->sp.B;
    for (int s = 0; s < nsub; ++s) {
      const Handle::SubStreams& ss = h->subs[s];
      SolveBlock& k = blk[s];
      const int b0 = (int)((int64_t)s * B / nsub), b1 = (int)((int64_t)(s + 1) * B / nsub);
      // the block's problems: gidx positions [b0, b1) (each group's range clipped to them);
      // the arrays stay the handle's (gidx holds absolute problem indices)
      k.sp = h->sp;
      for (int g = 0; g <= k.sp.ngrp; ++g) k.sp.go[g] = std::min(std::max(h->sp.go[g], b0), b1);
      k.d = h->d;
      k.s1 = ss.s1;
      k.s2 = ss.s2;
      k.fork = ss.fork;
      k.join = ss.join;
      k.s3 = ss.s3;
      k.pfork = ss.pfork;
      k.pjoin = ss.pjoin;
      HIPCHK(hipStreamWaitEvent(k.s1, h->evstart, 0));
    }
    // block s runs `lag` launches behind block s - 1 (its first launch waits on the gate
    // event recorded after launch lag - 1 of the block before; issued in that order)
    int lag = 1;
    if (const char* e = getenv("MHPC_SUB_LAG")) lag = atoi(e);  // tuning only
    lag = std::max(0, std::min(lag, nops - 1));
    // every block's streams are joined back to h->stream even when an issue fails partway,
    // so later work on the handle never races with a block's queued launches
    auto join_all = [&]() -> hipError_t {
      hipError_t e = hipSuccess;
      for (int s = 0; s < nsub; ++s) {
        hipError_t e1 = hipStreamWaitEvent(blk[s].s1, blk[s].join, 0);
        if (e1 == hipSuccess) e1 = hipEventRecord(h->subs[s].done, blk[s].s1);
        if (e1 == hipSuccess) e1 = hipStreamWaitEvent(h->stream, h->subs[s].done, 0);
        if (e == hipSuccess) e = e1;
      }
      return e;
    };
    rc = MHPC_OK;
    for (int t = 0; t < nops + (nsub - 1) * lag && !rc; ++t)
      for (int s = 0; s < nsub && !rc; ++s) {
        const int i = t - s * lag;
        if (i < 0 || i >= nops) continue;
        if (s > 0 && i == 0 && lag > 0 &&
            hipStreamWaitEvent(blk[s].s1, h->subs[s - 1].gate, 0) != hipSuccess)
          rc = fail(MHPC_ERR_DEVICE, "sub-batch gate wait failed");
        if (!rc) rc = issue_op(h, blk[s], ops[i]);
        if (!rc && s + 1 < nsub && lag > 0 && i == lag - 1 &&
            hipEventRecord(h->subs[s].gate, blk[s].s1) != hipSuccess)
          rc = fail(MHPC_ERR_DEVICE, "sub-batch gate record failed");
      }
    const hipError_t ej = join_all();
    if (rc) {  // (as above: the blocks' partials streams drained on an issue failure)
      for (int q = 0; q < nsub; ++q) {
        (void)hipStreamSynchronize(blk[q].s3);
        (void)hipStreamSynchronize(blk[q].s2);
      }
      return rc;
    }
    HIPCHK(ej);
  }
  // totals of the per-problem counters per layout group (tiny reduction, NCNT words each)
  HIPCHK(hipMemsetAsync(h->dcnt, 0, (size_t)h->sp.ngrp * NCNT * sizeof(unsigned long long), h->stream));
  HIPCHK(launch_reduce_counters(h->sp, h->d, h->dcnt, h->stream));
  return MHPC_OK;
}

int api_solve(Handle* h, int32_t* status) {
  if (!h) return fail(MHPC_ERR_INVALID, "null handle");
  if (!h->initialized) return fail(MHPC_ERR_STATE, "mhpc_initialize must precede mhpc_solve");
  if (h->solved) return fail(MHPC_ERR_STATE, "solve already ran: call mhpc_initialize or mhpc_update_problem");
  if (h->x0_changed)
    return fail(MHPC_ERR_STATE, "x0 changed: call mhpc_initialize or mhpc_update_problem first");
  if (h->params_changed)
    return fail(MHPC_ERR_STATE,
                "constraint parameters changed: call mhpc_initialize or mhpc_update_problem first");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipEventRecord(h->ev0, h->stream));
  int rc = solve_async(h);
  if (rc) return rc;
  HIPCHK(hipEventRecord(h->ev1, h->stream));
  HIPCHK(hipMemcpyAsync(h->gcnt, h->dcnt, (size_t)h->sp.ngrp * NCNT * sizeof(unsigned long long),
                        hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  for (int i = 0; i < NCNT; ++i) {
    h->cnt[i] = 0;
    for (int g = 0; g < h->sp.ngrp; ++g) h->cnt[i] += h->gcnt[g][i];
  }
  HIPCHK(hipEventElapsedTime(&h->solve_ms, h->ev0, h->ev1));
  h->solved = true;
  h->need_full = false;
  rc = collect_profile(h);
  if (rc) return rc;
  const unsigned long long* c = h->cnt;
  for (int g = 0; g < h->sp.ngrp; ++g) {  // per layout group: its problems' counters x its bytes
    const unsigned long long* cg = h->gcnt[g];
    const ByteModel& m = h->bym[g];
    const SolveParams& sp = h->sp;
    h->kbytes[K_FULL] += cg[C_FWD] * m.cost;
    // the trials that store their records (RO_STORE_FIRST; the re-rolls of the others, rare,
    // are not counted)
    const double stored = std::min(sp.n_cand, sp.ro_store + 1);
    h->kbytes[K_LS] += cg[C_LS_LAUNCH] * m.roll_read +
                       cg[C_LS_RUN] * (m.roll_write * stored / sp.n_cand + m.roll_term);
    h->kbytes[K_PAR] += cg[C_PAR_RUN] * m.par;
    h->kflops[K_LS] += cg[C_LS_RUN] * m.roll_flops;
  }
  // the SRB half of a split sweep: the SRB knots of every first attempt; the rest (WB knots,
  // impact steps, SRB knots of retries) is the WB half's / the whole sweep's
  const unsigned long long fb1 = c[C_BWS_KNOTS_FB1], fb = c[C_BWS_KNOTS_FB] - fb1;
  h->kbytes[K_BWS_SRB] += fb1 * kBwsFbKnot;
  h->kflops[K_BWS_SRB] += fb1 * kFlopFbKnot;
  h->kbytes[K_BWS] += c[C_BWS_KNOTS_WB] * kBwsWbKnot + fb * kBwsFbKnot + c[C_PX_READS] * kBwsPx;
  h->kflops[K_BWS] += c[C_BWS_KNOTS_WB] * kFlopWbKnot + fb * kFlopFbKnot + c[C_PX_READS] * kFlopPx;
  if (status) {
    std::vector<ProbState> st(h->sp.B);
    D2H(st.data(), h->d.st, st.size() * sizeof(ProbState));
    for (int b = 0; b < h->sp.B; ++b) status[b] = st[b].status;
  }
  return MHPC_OK;
}

// Rows [ko, ko + N) of a problem-major [B][NK][per] device array into buf ([B][N][per]):
// one strided copy of just the requested phase (not the whole trajectory buffer).
static int copy_rows(Handle* h, const real* src, int per, int ko, int N, size_t b0, size_t B,
                     std::vector<real>& buf) {
  const size_t NK = h->sp.NK, w = (size_t)N * per * sizeof(real);
  buf.resize(B * N * per);
  HIPCHK(hipMemcpy2DAsync(buf.data(), w, src + (b0 * NK + (size_t)ko) * per,
                          NK * per * sizeof(real), w, B, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return MHPC_OK;
}

// Problems [first, first + count) of one phase (count = batch: mhpc_get_phase).  The range's
// phase must have one shape (knots, state size); runs of problems whose phase starts at the
// same knot offset are copied with one strided copy each.
static int get_phase_run(Handle* h, int phase, int n, int N, int ko, size_t b0, size_t B, double* x,
                         double* u, double* y, double* K, double* du, double* Vx) {
  const SolveParams& sp = h->sp;
  std::vector<real> buf;
  int rc;
  if (x || u || y) {
    // export only the requested problems (a caller looping over problems would otherwise
    // export the whole batch per call)
    SolveParams sub = sp;
    sub.B = (int)B;
    HIPCHK(launch_export(sub, block_bufs(h->d, sp, b0), h->stream));
    if ((rc = copy_rows(h, h->d.out, KS, ko, N, b0, B, buf))) return rc;
    for (size_t b = 0; b < B; ++b)
      for (int k = 0; k < N; ++k) {
        const real* r = &buf[(b * N + k) * KS];
        for (int i = 0; i < n; ++i)
          if (x) x[(b * N + k) * n + i] = r[i];
        for (int i = 0; i < 4; ++i) {
          if (u) u[(b * N + k) * 4 + i] = r[n + i];
          if (y) y[(b * N + k) * 4 + i] = r[n + 4 + i];
        }
      }
  }
  if (K) {
    if ((rc = copy_rows(h, h->d.K, 56, ko, N, b0, B, buf))) return rc;
    for (size_t b = 0; b < B; ++b)
      for (int k = 0; k < N; ++k)
        for (int i = 0; i < 4 * n; ++i) K[(b * N + k) * 4 * n + i] = buf[(b * N + k) * 56 + i];
  }
  if (du) {
    if ((rc = copy_rows(h, h->d.du, 4, ko, N, b0, B, buf))) return rc;
    for (size_t i = 0; i < B * N * 4; ++i) du[i] = buf[i];
  }
  if (Vx) {
    if ((rc = copy_rows(h, h->d.G, 14, ko, N, b0, B, buf))) return rc;
    for (size_t b = 0; b < B; ++b)
      for (int k = 0; k < N; ++k)
        for (int i = 0; i < n; ++i) Vx[(b * N + k) * n + i] = buf[(b * N + k) * 14 + i];
  }
  return MHPC_OK;
}

// Shape check of a phase over a problem range: *n, *N of the phase (one shape for the range)
static int range_phase_shape(const Handle* h, int phase, int first, int count, int* n, int* N) {
  if (first < 0 || count < 1 || first > h->sp.B - count)
    return fail(MHPC_ERR_INVALID, "problem range outside the batch");
  for (int b = first; b < first + count; ++b) {
    const Layout& L = h->lays[h->lid[b]];
    if (phase < 0 || phase >= L.P) return fail(MHPC_ERR_INVALID, "bad phase");
    if (b == first) {
      *n = L.xs[phase];
      *N = L.N[phase];
    } else if (L.xs[phase] != *n || L.N[phase] != *N) {
      return fail(MHPC_ERR_INVALID, "the phase differs in shape across the problem range (per-problem layouts)");
    }
  }
  return MHPC_OK;
}

int api_get_phase(Handle* h, int phase, int first, int count, double* x, double* u, double* y,
                  double* K, double* du, double* Vx) {
  if (!h) return fail(MHPC_ERR_INVALID, "null handle");
  if (!h->initialized) return fail(MHPC_ERR_STATE, "not initialized");
  int n = 0, N = 0;
  int rc = range_phase_shape(h, phase, first, count, &n, &N);
  if (rc) return rc;
  HIPCHK(hipSetDevice(h->device));
  for (int r0 = first; r0 < first + count;) {
    const int ko = h->lays[h->lid[r0]].ko[phase];
    int r1 = r0 + 1;
    while (r1 < first + count && h->lays[h->lid[r1]].ko[phase] == ko) ++r1;
    const size_t o = (size_t)(r0 - first) * N;
    auto at = [&](double* p, int per) { return p ? p + o * per : nullptr; };
    rc = get_phase_run(h, phase, n, N, ko, r0, r1 - r0, at(x, n), at(u, 4), at(y, 4), at(K, 4 * n),
                       at(du, 4), at(Vx, n));
    if (rc) return rc;
    r0 = r1;
  }
  return MHPC_OK;
}

int api_get_scalars(Handle* h, double* J, double* dV_exp, double* viol,
                                double* V_phase, double* dV_phase, int32_t* trace) {
  if (!h) return fail(MHPC_ERR_INVALID, "null handle");
  if (!h->initialized) return fail(MHPC_ERR_STATE, "not initialized");
  HIPCHK(hipSetDevice(h->device));
  const SolveParams& sp = h->sp;
  std::vector<ProbState> st(sp.B);
  D2H(st.data(), h->d.st, st.size() * sizeof(ProbState));
  for (int b = 0; b < sp.B; ++b) {
    if (J) J[b] = st[b].J;
    if (dV_exp) dV_exp[b] = st[b].dV_exp;
    if (viol) viol[b] = st[b].viol;
    // rows of the most phases any layout has; zero past the problem's own phases
    const int P = h->lays[h->lid[b]].P;
    for (int p = 0; p < sp.pmax; ++p) {
      if (V_phase) V_phase[b * sp.pmax + p] = p < P ? (double)st[b].V[p] : 0.0;
      if (dV_phase) dV_phase[b * sp.pmax + p] = p < P ? (double)st[b].dV[p] : 0.0;
    }
    if (trace) memcpy(&trace[(size_t)b * TRACE], st[b].trace, TRACE * sizeof(int32_t));
  }
  return MHPC_OK;
}

int api_rollout_costs(Handle* h, int n_eps, const double* eps, double* J,
                                  double* viol, float* ms) {
  if (!h || !eps || !J) return fail(MHPC_ERR_INVALID, "null argument");
  if (!h->initialized) return fail(MHPC_ERR_STATE, "not initialized");
  if (n_eps < 1 || n_eps > MHPC_MAX_ROLLOUT_EPS) return fail(MHPC_ERR_INVALID, "n_eps out of range");
  HIPCHK(hipSetDevice(h->device));
  const size_t B = h->sp.B, n = B * (size_t)n_eps;
  real *deps = nullptr, *dJ = nullptr, *dv = nullptr;
  std::vector<real> heps(eps, eps + n_eps), hJ(n), hv(n);
  auto cleanup = [&]() {
    if (deps) (void)hipFree(deps);
    if (dJ) (void)hipFree(dJ);
    if (dv) (void)hipFree(dv);
  };
  hipError_t e = hipMalloc((void**)&deps, n_eps * sizeof(real));
  if (e == hipSuccess) e = hipMalloc((void**)&dJ, n * sizeof(real));
  if (e == hipSuccess) e = hipMalloc((void**)&dv, n * sizeof(real));
  if (e == hipSuccess) e = hipMemcpyAsync(deps, heps.data(), n_eps * sizeof(real), hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) e = hipEventRecord(h->ev0, h->stream);
  if (e == hipSuccess) e = launch_eps_rollout(h->sp, h->d, n_eps, deps, dJ, dv, h->stream);
  if (e == hipSuccess) e = hipEventRecord(h->ev1, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(hJ.data(), dJ, n * sizeof(real), hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(hv.data(), dv, n * sizeof(real), hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e == hipSuccess)
    for (size_t i = 0; i < n; ++i) {
      J[i] = hJ[i];
      if (viol) viol[i] = hv[i];
    }
  float t = 0;
  if (e == hipSuccess) e = hipEventElapsedTime(&t, h->ev0, h->ev1);
  cleanup();
  if (e != hipSuccess) return fail(MHPC_ERR_DEVICE, std::string("mhpc_rollout_costs: ") + hipGetErrorString(e));
  if (ms) *ms = t;
  return MHPC_OK;
}

int api_get_cost_gradients(Handle* h, int phase, int first, int count, double* lx, double* Phix) {
  if (!h) return fail(MHPC_ERR_INVALID, "null handle");
  if (!h->initialized) return fail(MHPC_ERR_STATE, "not initialized");
  const SolveParams& sp = h->sp;
  int n = 0, N = 0;
  int rc = range_phase_shape(h, phase, first, count, &n, &N);
  if (rc) return rc;
  HIPCHK(hipSetDevice(h->device));
  const size_t nlx = (size_t)count * (N - 1) * n, nph = (size_t)count * n;
  real *dlx = nullptr, *dph = nullptr;
  std::vector<real> hlx(nlx), hph(nph);
  hipError_t e = hipMalloc((void**)&dlx, nlx * sizeof(real) + 8);
  if (e == hipSuccess) e = hipMalloc((void**)&dph, nph * sizeof(real));
  // one launch per run of problems with the same layout
  for (int r0 = first; r0 < first + count && e == hipSuccess;) {
    const int g = h->lid[r0];
    int r1 = r0 + 1;
    while (r1 < first + count && h->lid[r1] == g) ++r1;
    const size_t o = (size_t)(r0 - first);
    e = launch_cost_grad(sp, h->d, g, phase, N, r0, r1 - r0, dlx + o * (N - 1) * n, dph + o * n,
                         h->stream);
    r0 = r1;
  }
  if (e == hipSuccess) e = hipMemcpyAsync(hlx.data(), dlx, nlx * sizeof(real), hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(hph.data(), dph, nph * sizeof(real), hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e == hipSuccess) {
    if (lx) std::copy(hlx.begin(), hlx.end(), lx);
    if (Phix) std::copy(hph.begin(), hph.end(), Phix);
  }
  if (dlx) (void)hipFree(dlx);
  if (dph) (void)hipFree(dph);
  if (e != hipSuccess) return fail(MHPC_ERR_DEVICE, std::string("mhpc_get_cost_gradients: ") + hipGetErrorString(e));
  return MHPC_OK;
}

// The phase-buffer store of the receding-horizon loop, [B][spmax][nbk][SREC], zeroed at its
// first use after an initialize (the reference's memory_reset of its phase buffers); sized for
// the current layouts (buffers of N_TIMESTEPS_MAX = 110 knots, or the longest phase).
static int ensure_store(Handle* h) {
  if (h->store_valid) return MHPC_OK;
  int nbk = kPhaseBufKnots;
  for (const Layout& L : h->lays)
    for (int p = 0; p < L.P; ++p) nbk = std::max(nbk, L.N[p]);
  const int spmax = h->sp.pmax;
  const size_t bytes = (size_t)h->sp.B * spmax * nbk * kStoreRec * sizeof(real);
  if (!h->store || nbk != h->nbk || spmax != h->spmax) {
    if (h->store) HIPCHK(hipFree(h->store));
    h->store = nullptr;
    HIPCHK(hipMalloc((void**)&h->store, bytes));
    h->nbk = nbk;
    h->spmax = spmax;
  }
  HIPCHK(hipMemsetAsync(h->store, 0, bytes, h->stream));
  h->store_valid = true;
  return MHPC_OK;
}

// MHPCLocomotion::update_problem (MHPCLocomotion.cpp:107-158) per problem: problem b takes
// steps[b] gait steps (each: rotate the WB and SRB phase buffers by one, advance the gait by
// one mode, recompute mode sequence and knot counts -- Gait.h:48-77); then every problem's
// references are regenerated from the current x0 (mhpc_set_x0) and its AL / ReB parameters
// re-initialised.  The rotated nominal trajectories and gains are the warm start of the next
// mhpc_solve, whose first forward_sweep(0) is then a real rollout.  Problems whose layouts
// change move to the layout group of their new layout.
int api_update_problems(Handle* h, int n_gaits, const mhpc_gait* gaits, const int32_t* gait_of,
                        const int32_t* steps) {
  if (!h || !gaits) return fail(MHPC_ERR_INVALID, "null argument");
  if (!h->initialized) return fail(MHPC_ERR_STATE, "mhpc_initialize must precede mhpc_update_problem");
  if (n_gaits < 1 || n_gaits > MAXL) return fail(MHPC_ERR_INVALID, "n_gaits must be 1..MHPC_MAX_LAYOUTS");
  for (int gi = 0; gi < n_gaits; ++gi) {
    const mhpc_gait& g = gaits[gi];
    if (g.n_modes < 1 || g.n_modes > MHPC_MAX_PHASES)
      return fail(MHPC_ERR_INVALID, "gait needs 1..16 modes");
    for (int i = 0; i < g.n_modes; ++i)
      if (g.modes[i] < 1 || g.modes[i] > 4) return fail(MHPC_ERR_INVALID, "gait mode out of range");
  }
  HIPCHK(hipSetDevice(h->device));
  int rc = ensure_store(h);
  if (rc) return rc;
  const int B = h->sp.B;
  std::vector<ProbLayout> npl = h->pl;
  std::vector<int> ncm = h->cmode;
  for (int b = 0; b < B; ++b) {
    const int gi = gait_of ? gait_of[b] : 0;
    if (gi < 0 || gi >= n_gaits) return fail(MHPC_ERR_INVALID, "gait index out of range");
    const int ns = steps ? steps[b] : 1;
    if (ns < 0 || ns > 1024) return fail(MHPC_ERR_INVALID, "steps must be 0..1024");
    const mhpc_gait& gait = gaits[gi];
    // Gait::get_next_mode / get_mode_seq / get_timings (Gait.h:48-77)
    auto next_mode = [&](int m) {
      for (int i = 0; i < gait.n_modes; ++i)
        if (gait.modes[i] == m) return gait.modes[(i + 1) % gait.n_modes];
      return -1;  // the reference falls off the end of a non-void function here
    };
    mhpc_problem_desc& nd = npl[b].desc;
    const int P = nd.n_wb + nd.n_fb;
    for (int step = 0; step < ns; ++step) {
      const int cm = next_mode(ncm[b]);
      if (cm < 0) return fail(MHPC_ERR_INVALID, "current mode is not in the gait");
      ncm[b] = cm;
      nd.mode_seq[0] = cm;
      for (int p = 1; p < P; ++p) nd.mode_seq[p] = next_mode(nd.mode_seq[p - 1]);
      int NK = 0;
      for (int p = 0; p < P; ++p) {
        const float tm = gait.timings[nd.mode_seq[p] - 1];
        const double dt = p < nd.n_wb ? nd.dt_wb : nd.dt_fb;
        nd.N[p] = (int)std::round((double)tm / dt);  // round(float timing / (double) dt)
        if (nd.N[p] < 2) return fail(MHPC_ERR_INVALID, "gait timing gives a phase with N < 2");
        if (nd.N[p] > h->nbk) return fail(MHPC_ERR_INVALID, "phase longer than the phase buffers");
        NK += nd.N[p];
      }
      if (NK > MHPC_MAX_KNOTS) return fail(MHPC_ERR_INVALID, "too many knots");
      // pidx_WB / pidx_FB: front -> back (MHPCLocomotion.cpp:111-121); kept reduced, so a
      // long receding-horizon loop never overflows the count
      npl[b].rot_wb = (npl[b].rot_wb + 1) % std::max(nd.n_wb, 1);
      npl[b].rot_fb = (npl[b].rot_fb + 1) % std::max(nd.n_fb, 1);
    }
  }
  // phases write through to their buffers in the reference: save the current layouts
  HIPCHK(launch_store(h->sp, h->d, h->store, h->nbk, h->spmax, 1, h->stream));
  const std::vector<ProbLayout> opl = h->pl;
  h->pl = npl;
  if ((rc = rebuild_groups(h))) {  // too many distinct layouts: keep the old ones
    h->pl = opl;
    (void)rebuild_groups(h);
    return rc;
  }
  h->cmode = ncm;
  HIPCHK(launch_reset(h->sp, h->d, h->stream));  // refs from x0, AL/ReB init, nom_slot = 0
  HIPCHK(launch_store(h->sp, h->d, h->store, h->nbk, h->spmax, 0, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  h->need_full = true;
  h->solved = false;
  h->x0_changed = false;
  h->params_changed = false;
  return MHPC_OK;
}

int api_update_problem(Handle* h, const mhpc_gait* gait) {
  return api_update_problems(h, 1, gait, nullptr, nullptr);
}

// Per-problem phase layouts (the batch axis over gait schedules): problem b gets
// descs[lop[b]] with identity phase buffers; the handle is uninitialised afterwards.
int api_set_layouts(Handle* h, int n_desc, const mhpc_problem_desc* descs, const int32_t* lop) {
  if (!h || !descs) return fail(MHPC_ERR_INVALID, "null argument");
  if (n_desc < 1 || n_desc > MAXL) return fail(MHPC_ERR_INVALID, "n_desc must be 1..MHPC_MAX_LAYOUTS");
  for (int i = 0; i < n_desc; ++i) {
    int rc = validate(&descs[i]);
    if (rc) return rc;
    if (descs[i].precision != h->desc.precision)
      return fail(MHPC_ERR_INVALID, "a layout's precision differs from the handle's");
    if (descs[i].vel_cmd != h->desc.vel_cmd || descs[i].height_cmd != h->desc.height_cmd)
      return fail(MHPC_ERR_INVALID, "a layout's vel_cmd / height_cmd differs from the handle's");
  }
  const int B = h->sp.B;
  for (int b = 0; lop && b < B; ++b)
    if (lop[b] < 0 || lop[b] >= n_desc) return fail(MHPC_ERR_INVALID, "layout index out of range");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize(h->stream));
  const std::vector<ProbLayout> opl = h->pl;
  for (int b = 0; b < B; ++b) {
    const mhpc_problem_desc& d = descs[lop ? lop[b] : b % n_desc];
    h->pl[b] = ProbLayout{norm_desc(d), 0, 0};
  }
  int rc = rebuild_groups(h);
  if (rc) {
    h->pl = opl;
    (void)rebuild_groups(h);
    return rc;
  }
  for (int b = 0; b < B; ++b) h->cmode[b] = h->pl[b].desc.mode_seq[0];
  h->store_valid = false;
  h->initialized = false;
  h->solved = false;
  h->x0_set = false;  // the x0 row length may have changed
  return MHPC_OK;
}

int api_get_problem_desc(Handle* h, int b, mhpc_problem_desc* desc) {
  if (!h || !desc) return fail(MHPC_ERR_INVALID, "null argument");
  if (b < 0 || b >= h->sp.B) return fail(MHPC_ERR_INVALID, "problem out of range");
  *desc = h->pl[b].desc;
  return MHPC_OK;
}

int api_num_layouts(Handle* h, int* n) {
  if (!h || !n) return fail(MHPC_ERR_INVALID, "null argument");
  *n = h->sp.ngrp;
  return MHPC_OK;
}

// the row length of get_scalars' V_phase / dV_phase (rebuild_groups: sp.pmax)
int api_max_phases(Handle* h, int* n) {
  if (!h || !n) return fail(MHPC_ERR_INVALID, "null argument");
  *n = h->sp.pmax;
  return MHPC_OK;
}

int api_batch(Handle* h) { return h ? h->sp.B : 0; }

int api_get_desc(Handle* h, mhpc_problem_desc* desc) {
  if (!h || !desc) return fail(MHPC_ERR_INVALID, "null argument");
  *desc = h->pl[0].desc;
  return MHPC_OK;
}

int api_get_counters(Handle* h, mhpc_counters* c) {
  if (!h || !c) return fail(MHPC_ERR_INVALID, "null argument");
  memset(c, 0, sizeof *c);
  c->ddp_iters = (int64_t)h->cnt[C_DDP];
  c->bws_sweeps = (int64_t)h->cnt[C_BWS];
  c->bws_knots = (int64_t)h->cnt[C_BWS_KNOTS];
  c->ls_rollouts = (int64_t)h->cnt[C_LS];
  c->fwd_sweeps = (int64_t)h->cnt[C_FWD];
  c->partial_sweeps = (int64_t)h->cnt[C_PAR];
  c->solve_ms = h->solve_ms;
  return MHPC_OK;
}

int api_set_profiling(Handle* h, int on) {
  if (!h) return fail(MHPC_ERR_INVALID, "null handle");
  h->profile = on != 0;
  return MHPC_OK;
}

int api_get_kernel_stats(Handle* h, double* ms, int64_t* launches,
                                     double* alg_bytes) {
  if (!h) return fail(MHPC_ERR_INVALID, "null handle");
  for (int k = 0; k < NKERN; ++k) {
    if (ms) ms[k] = h->kms[k];
    if (launches) launches[k] = h->klaunch[k];
    if (alg_bytes) alg_bytes[k] = h->kbytes[k];
  }
  return MHPC_OK;
}

int api_set_kernel_variant(Handle* h, int which, int variant) {
  if (!h) return fail(MHPC_ERR_INVALID, "null handle");
  SolveParams& sp = h->sp;
  if (which == MHPC_VARIANT_BWS) {
    if (variant < 0 || variant > MHPC_VARIANT_BWS_PAIRS2) return fail(MHPC_ERR_INVALID, "no such backward-sweep variant");
    sp.var_bws = variant;
    return MHPC_OK;
  }
  if (which == MHPC_VARIANT_OVERLAP) {
    if (variant < 0 || variant > MHPC_VARIANT_OVERLAP_OFF) return fail(MHPC_ERR_INVALID, "no such overlap variant");
    sp.var_overlap = variant;
    return MHPC_OK;
  }
  if (which == MHPC_VARIANT_RO_STORE) {
    if (variant < 0 || variant > MAXC) return fail(MHPC_ERR_INVALID, "stored trials must be 0..32");
    h->ro_store_req = variant;
    sp.ro_store = variant ? variant : ro_store_auto(sp);
    return MHPC_OK;
  }
  if (which == MHPC_VARIANT_SWEEP_BITS) {
    if (variant != 0 && variant != 64 && !(variant == 32 && sizeof(real) == 4))
      return fail(MHPC_ERR_INVALID, "sweep arithmetic must be 0 / 64 (double), or 32 (float) in an fp32 handle");
    h->sweep_bits = variant;
    return MHPC_OK;
  }
  if (which == MHPC_VARIANT_SUBBATCH) {
    if (variant < 0 || variant > MHPC_MAX_SUBBATCH) return fail(MHPC_ERR_INVALID, "sub-batch count must be 0..4");
    h->nsub_req = variant;
    return MHPC_OK;
  }
  if (which != MHPC_VARIANT_RO) return fail(MHPC_ERR_INVALID, "no such kernel");
  if (variant < 0 || variant > MHPC_VARIANT_RO_FUSED) return fail(MHPC_ERR_INVALID, "no such line-search variant");
  const bool staged = variant == MHPC_VARIANT_RO_PAIR || variant == MHPC_VARIANT_RO_PIPE_STAGED ||
                      variant == MHPC_VARIANT_RO_FUSED_STAGED;
  if (staged && 64 / sp.n_cand > 6)  // ST_PPW problems per staged wave (mhpc_kernels.hip)
    return fail(MHPC_ERR_INVALID, "staged line-search variants need >= 10 candidates");
  if (variant == MHPC_VARIANT_RO_PAIR && 32 / sp.n_cand < 1)
    return fail(MHPC_ERR_INVALID, "the pair variant needs <= 32 candidates");
  sp.var_ro = variant;
  return MHPC_OK;
}

int api_get_kernel_flops(Handle* h, double* flops) {
  if (!h || !flops) return fail(MHPC_ERR_INVALID, "null argument");
  for (int k = 0; k < NKERN; ++k) flops[k] = h->kflops[k];
  return MHPC_OK;
}

int api_reset_kernel_stats(Handle* h) {
  if (!h) return fail(MHPC_ERR_INVALID, "null handle");
  for (int k = 0; k < NKERN; ++k) {
    h->kms[k] = 0; h->kbytes[k] = 0; h->kflops[k] = 0; h->klaunch[k] = 0;
  }
  return MHPC_OK;
}

void api_destroy(Handle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  // every stream of the handle drains before its buffers go (an error inside a solve can
  // leave work queued on the partials' or a sub-batch's streams)
  for (hipStream_t q : {h->stream, h->stream2, h->stream3})
    if (q) (void)hipStreamSynchronize(q);
  for (Handle::SubStreams& s : h->subs)
    for (hipStream_t q : {s.s1, s.s2, s.s3})
      if (q) (void)hipStreamSynchronize(q);
  free_bufs(h);
  if (h->dcnt) (void)hipFree(h->dcnt);
  if (h->store) (void)hipFree(h->store);
  for (hipEvent_t e : h->evpool) (void)hipEventDestroy(e);
  if (h->ev0) (void)hipEventDestroy(h->ev0);
  if (h->ev1) (void)hipEventDestroy(h->ev1);
  if (h->evfork) (void)hipEventDestroy(h->evfork);
  if (h->evjoin) (void)hipEventDestroy(h->evjoin);
  if (h->stream2) (void)hipStreamDestroy(h->stream2);
  if (h->stream3) (void)hipStreamDestroy(h->stream3);
  if (h->evpfork) (void)hipEventDestroy(h->evpfork);
  if (h->evpjoin) (void)hipEventDestroy(h->evpjoin);
  for (Handle::SubStreams& s : h->subs) {
    for (hipStream_t q : {s.s1, s.s2, s.s3})
      if (q) (void)hipStreamDestroy(q);
    for (hipEvent_t e : {s.fork, s.join, s.gate, s.done, s.pfork, s.pjoin})
      if (e) (void)hipEventDestroy(e);
  }
  if (h->evstart) (void)hipEventDestroy(h->evstart);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

#ifndef MHPC_FP32  // kernel-level parity hooks: fp64 only
// ---- batched model evaluation hooks ---------------------------------------------------------
namespace {
struct DevScratch {
  std::vector<void*> ptrs;
  ~DevScratch() {
    for (void* p : ptrs) (void)hipFree(p);
  }
  double* put(const double* host, size_t n, hipError_t* e) {
    void* p = nullptr;
    if (*e == hipSuccess) *e = hipMalloc(&p, n * sizeof(double) + 8);
    if (*e == hipSuccess) ptrs.push_back(p);
    if (*e == hipSuccess && host) *e = hipMemcpy(p, host, n * sizeof(double), hipMemcpyHostToDevice);
    return (double*)p;
  }
};
}  // namespace

extern "C" int mhpc_eval_wb_dynamics(int device, int n, int mode, const double* x, const double* u,
                                     double* xdot, double* y) {
  if (n < 1 || !x || !u || !xdot || !y || mode < 1 || mode > 4)
    return fail(MHPC_ERR_INVALID, "bad argument");
  HIPCHK(hipSetDevice(device));
  DevScratch s;
  hipError_t e = hipSuccess;
  double *dx = s.put(x, n * 14, &e), *du = s.put(u, n * 4, &e);
  double *dxd = s.put(nullptr, n * 14, &e), *dy = s.put(nullptr, n * 4, &e);
  HIPCHK(e);
  HIPCHK(launch_eval_wb_dyn(n, mode, dx, du, dxd, dy, nullptr));
  HIPCHK(hipMemcpy(xdot, dxd, n * 14 * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(y, dy, n * 4 * sizeof(double), hipMemcpyDeviceToHost));
  return MHPC_OK;
}

extern "C" int mhpc_eval_wb_dynamics_pair(int device, int n, int mode, const double* x,
                                          const double* u, double* xdot, double* y) {
  if (n < 1 || !x || !u || !xdot || !y || mode < 1 || mode > 4)
    return fail(MHPC_ERR_INVALID, "bad argument");
  HIPCHK(hipSetDevice(device));
  DevScratch s;
  hipError_t e = hipSuccess;
  double *dx = s.put(x, n * 14, &e), *du = s.put(u, n * 4, &e);
  double *dxd = s.put(nullptr, n * 28, &e), *dy = s.put(nullptr, n * 8, &e);
  HIPCHK(e);
  HIPCHK(launch_eval_wb_dyn_pair(n, mode, dx, du, dxd, dy, nullptr));
  HIPCHK(hipMemcpy(xdot, dxd, n * 28 * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(y, dy, n * 8 * sizeof(double), hipMemcpyDeviceToHost));
  return MHPC_OK;
}

extern "C" int mhpc_eval_wb_touchdown(int device, int n, int foot, const double* x, double* h,
                                      double* hx, double* hxx, double* J, double* Jd) {
  if (n < 1 || !x || !h || !hx || !hxx || !J || !Jd || (foot != 0 && foot != 1))
    return fail(MHPC_ERR_INVALID, "bad argument");
  HIPCHK(hipSetDevice(device));
  DevScratch s;
  hipError_t e = hipSuccess;
  double *dx = s.put(x, n * 14, &e), *dh = s.put(nullptr, n * 2, &e);
  double *dhx = s.put(nullptr, n * 14, &e), *dhxx = s.put(nullptr, n * 196, &e);
  double *dJ = s.put(nullptr, n * 14, &e), *dJd = s.put(nullptr, n * 14, &e);
  HIPCHK(e);
  HIPCHK(launch_eval_wb_aux(n, foot, dx, dh, dhx, dhxx, dJ, dJd, nullptr));
  HIPCHK(hipMemcpy(h, dh, n * 2 * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(hx, dhx, n * 14 * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(hxx, dhxx, n * 196 * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(J, dJ, n * 14 * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(Jd, dJd, n * 14 * sizeof(double), hipMemcpyDeviceToHost));
  return MHPC_OK;
}

extern "C" int mhpc_eval_wb_partials(int device, int n, int mode, const double* x, const double* u,
                                     double* Ac, double* Bc, double* C, double* D) {
  if (n < 1 || !x || !u || !Ac || !Bc || !C || !D || mode < 1 || mode > 4)
    return fail(MHPC_ERR_INVALID, "bad argument");
  HIPCHK(hipSetDevice(device));
  DevScratch s;
  hipError_t e = hipSuccess;
  double *dx = s.put(x, n * 14, &e), *du = s.put(u, n * 4, &e);
  double *dA = s.put(nullptr, n * 196, &e), *dB = s.put(nullptr, n * 56, &e);
  double *dC = s.put(nullptr, n * 56, &e), *dD = s.put(nullptr, n * 16, &e);
  HIPCHK(e);
  HIPCHK(launch_eval_wb_par(n, mode, dx, du, dA, dB, dC, dD, nullptr));
  HIPCHK(hipMemcpy(Ac, dA, n * 196 * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(Bc, dB, n * 56 * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(C, dC, n * 56 * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(D, dD, n * 16 * sizeof(double), hipMemcpyDeviceToHost));
  return MHPC_OK;
}

extern "C" int mhpc_eval_wb_impact(int device, int n, int foot, const double* x, double* xplus,
                                   double* Px) {
  if (n < 1 || !x || !xplus || !Px || (foot != 0 && foot != 1))
    return fail(MHPC_ERR_INVALID, "bad argument");
  HIPCHK(hipSetDevice(device));
  DevScratch s;
  hipError_t e = hipSuccess;
  double *dx = s.put(x, n * 14, &e), *dxp = s.put(nullptr, n * 14, &e);
  double* dP = s.put(nullptr, n * 196, &e);
  HIPCHK(e);
  HIPCHK(launch_eval_wb_impact(n, foot, dx, dxp, dP, nullptr));
  HIPCHK(hipMemcpy(xplus, dxp, n * 14 * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(Px, dP, n * 196 * sizeof(double), hipMemcpyDeviceToHost));
  return MHPC_OK;
}

extern "C" int mhpc_eval_srb(int device, int n, const double* x, const double* u,
                             const double* foothold, const double* contact, double* xdot,
                             double* Ac, double* Bc) {
  if (n < 1 || !x || !u || !foothold || !contact || !xdot || !Ac || !Bc)
    return fail(MHPC_ERR_INVALID, "bad argument");
  HIPCHK(hipSetDevice(device));
  DevScratch s;
  hipError_t e = hipSuccess;
  double *dx = s.put(x, n * 6, &e), *du = s.put(u, n * 4, &e), *dp = s.put(foothold, n * 4, &e);
  double *dc = s.put(contact, n * 2, &e), *dxd = s.put(nullptr, n * 6, &e);
  double *dA = s.put(nullptr, n * 36, &e), *dB = s.put(nullptr, n * 24, &e);
  HIPCHK(e);
  HIPCHK(launch_eval_srb(n, dx, du, dp, dc, dxd, dA, dB, nullptr));
  HIPCHK(hipMemcpy(xdot, dxd, n * 6 * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(Ac, dA, n * 36 * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(Bc, dB, n * 24 * sizeof(double), hipMemcpyDeviceToHost));
  return MHPC_OK;
}
#else   // MHPC_FP32: the fp32 build of the two rollout dynamics models
// Whole-body dynamics of the fp32 instantiation, single-lane (pair = 0: xdot [n][14],
// y [n][4]) or lane pair (pair = 1: xdot [n][2][14], y [n][2][4]); host arrays double.
extern "C" int mhpc_eval_wb_dynamics_f32(int device, int n, int mode, int pair, const double* x,
                                         const double* u, double* xdot, double* y) {
  if (n < 1 || !x || !u || !xdot || !y || mode < 1 || mode > 4 || (pair != 0 && pair != 1))
    return fail(MHPC_ERR_INVALID, "bad argument");
  HIPCHK(hipSetDevice(device));
  const int L = pair ? 2 : 1;
  std::vector<float> hx(x, x + (size_t)n * 14), hu(u, u + (size_t)n * 4);
  std::vector<float> hxd((size_t)n * 14 * L), hy((size_t)n * 4 * L);
  float *dx = nullptr, *du = nullptr, *dxd = nullptr, *dy = nullptr;
  hipError_t e = hipMalloc((void**)&dx, hx.size() * 4);
  if (e == hipSuccess) e = hipMalloc((void**)&du, hu.size() * 4);
  if (e == hipSuccess) e = hipMalloc((void**)&dxd, hxd.size() * 4);
  if (e == hipSuccess) e = hipMalloc((void**)&dy, hy.size() * 4);
  if (e == hipSuccess) e = hipMemcpy(dx, hx.data(), hx.size() * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(du, hu.data(), hu.size() * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = pair ? launch_eval_wb_dyn_pair(n, mode, dx, du, dxd, dy, nullptr)
             : launch_eval_wb_dyn(n, mode, dx, du, dxd, dy, nullptr);
  if (e == hipSuccess) e = hipMemcpy(hxd.data(), dxd, hxd.size() * 4, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(hy.data(), dy, hy.size() * 4, hipMemcpyDeviceToHost);
  for (float* p : {dx, du, dxd, dy})
    if (p) (void)hipFree(p);
  if (e != hipSuccess) return fail(MHPC_ERR_DEVICE, std::string("mhpc_eval_wb_dynamics_f32: ") + hipGetErrorString(e));
  std::copy(hxd.begin(), hxd.end(), xdot);
  std::copy(hy.begin(), hy.end(), y);
  return MHPC_OK;
}
#endif  // MHPC_FP32

}  // namespace MHPC_NS
