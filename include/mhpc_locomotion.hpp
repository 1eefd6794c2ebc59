// mhpc_locomotion.hpp -- C++ host surface of the reference controller over the C-ABI.
//
// Same names, fields and defaults as the reference's API so that the reference's driver
// (test_main.cpp:12-35) compiles against it unchanged except for the include:
//   HSDDP_OPTION<T>        MHPC_CompoundTypes.h:196-212
//   USRCMD                 MHPC_CompoundTypes.h:237-240
//   MHPCUserParameters     MHPC_CompoundTypes.h:242-251  (alias MHPC_UserParameter)
//   GaitType2D, Gait       Gait.h:6-77
//   MHPCLocomotion<T>      MHPCLocomotion.h:13-83 (initialization, solve_mhpc, print_debugInfo)
//   MultiPhaseDDP<T>       MultiPhaseDDP.h:12-63 (public _phases, _n_phases, _option,
//                          _actual_cost, _exp_cost_change, _tconstr_violation)
//   SinglePhaseAbstract<T> SinglePhaseAbstract.h:66-134 (public _modeidx, _phaseidx, _dt,
//                          _N_TIMESTEPS, _V, _dV, _xsize/_usize/_ysize, get_modeidx,
//                          get_nominal_ms_ptr, get_CTG_info_ptr, get_terminal_state)
//   ModelState, CostToGoStruct  MHPC_CompoundTypes.h:7-22,88-114 (x/u/y; G, du, K)
// The heavy lifting happens in libmhpc_amd.so (HIP, gfx950).  Extensions: a batch of
// independent problems per object, and set_initial_conditions() for per-problem x0.
// Header-only; link with -lmhpc_amd.  Errors throw std::runtime_error on this side of
// the ABI (none cross it).
#pragma once
#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "mhpc_capi.h"

template <typename T>
struct HSDDP_OPTION {
  T alpha = 0.1;
  T gamma = 0.01;
  T update_penalty = 8;
  T update_relax = 0.1;
  T update_regularization = 2;
  T update_ReB = 7;
  T max_DDP_iter = 3;
  T max_AL_iter = 2;
  T DDP_thresh = 1e-03;
  T AL_thresh = 1e-03;
  bool AL_active = 1;
  bool ReB_active = 1;
  bool smooth_active = 0;
};

struct USRCMD {
  float vel, height, roll, pitch, yaw;
};

struct MHPCUserParameters {
  int n_wbphase = 4;
  int n_fbphase = 4;
  float dt_wb = .001;
  float dt_fb = .001;
  int cmode = 1;
  float groundH = -0.404;  // unused, as in the reference (ground hard-coded at -0.404)
  USRCMD* usrcmd = nullptr;
};
using MHPC_UserParameter = MHPCUserParameters;

enum class GaitType2D { STAND, BOUND, PRONK };

class Gait {
 public:
  Gait() : mode_{1, 2, 3, 4}, timing_{0.08f, 0.1f, 0.08f, 0.1f} {}
  explicit Gait(GaitType2D g) : mode_{1, 2, 3, 4} {
    if (g == GaitType2D::BOUND) timing_ = {0.08f, 0.1f, 0.08f, 0.1f};
    else timing_ = {0.08f, 0.08f, 0.08f, 0.08f};  // default branch of the reference switch
  }
  int get_next_mode(int current_mode) const {
    for (size_t i = 0; i < mode_.size(); ++i)
      if (mode_[i] == current_mode) return mode_[(i + 1) % mode_.size()];
    throw std::runtime_error("mode not in gait");
  }
  std::vector<int> get_mode_seq(int current_mode, int num_phases) const {
    std::vector<int> s(num_phases);
    s[0] = current_mode;
    for (int p = 0; p + 1 < num_phases; ++p) s[p + 1] = get_next_mode(s[p]);
    return s;
  }
  std::vector<float> get_timings(const std::vector<int>& seq) const {
    std::vector<float> t(seq.size());
    for (size_t i = 0; i < seq.size(); ++i) t[i] = timing_[seq[i] - 1];
    return t;
  }
  mhpc_gait to_c() const {
    mhpc_gait g{};
    g.n_modes = (int)mode_.size();
    for (size_t i = 0; i < mode_.size(); ++i) g.modes[i] = mode_[i];
    for (size_t i = 0; i < timing_.size(); ++i) g.timings[i] = timing_[i];
    return g;
  }

 private:
  std::vector<int> mode_;
  std::vector<float> timing_;
};

// Fixed-size vector / matrix with Eigen's element access (v(i), v[i], m(r, c); m stored
// column-major like Eigen's default), enough for reading solver output the way the
// reference's callers read VecM / MatMN (MHPC_CPPTypes.h).
template <typename T, size_t n>
struct VecM {
  T v[n] = {};
  T& operator()(size_t i) { return v[i]; }
  const T& operator()(size_t i) const { return v[i]; }
  T& operator[](size_t i) { return v[i]; }
  const T& operator[](size_t i) const { return v[i]; }
  static constexpr size_t size() { return n; }
  T* data() { return v; }
  const T* data() const { return v; }
};
template <typename T, size_t r, size_t c>
struct MatMN {
  T v[r * c] = {};
  T& operator()(size_t i, size_t j) { return v[j * r + i]; }
  const T& operator()(size_t i, size_t j) const { return v[j * r + i]; }
  static constexpr size_t rows() { return r; }
  static constexpr size_t cols() { return c; }
  T* data() { return v; }
  const T* data() const { return v; }
};

// One knot of a phase's nominal trajectory (MHPC_CompoundTypes.h:7-22)
template <typename T, size_t xsize, size_t usize, size_t ysize>
struct ModelState {
  VecM<T, xsize> x;
  VecM<T, usize> u;
  VecM<T, ysize> y;
};

// One knot of a phase's cost-to-go information (MHPC_CompoundTypes.h:88-101): the value
// gradient G (Vx) and the feedback du, K that the execution horizon consumes.  The Hessian H
// and the Q-function blocks are intermediates of the backward sweep that the device keeps
// in LDS and never writes to HBM; they are not part of this struct (reading them fails to
// compile instead of returning zeros).
template <typename T, size_t xsize, size_t usize>
struct CostToGoStruct {
  VecM<T, xsize> G;
  VecM<T, usize> du;
  MatMN<T, usize, xsize> K;
};

// Read-only view of one phase of one problem of the batch after a solve, with the public
// members and accessors of the reference's SinglePhaseAbstract (SinglePhaseAbstract.h:66-134).
// The nominal / cost-to-go arrays are copied from the device on first access after a solve.
template <typename T>
class SinglePhaseAbstract {
 public:
  int _modeidx = 1;
  int _phaseidx = 1;
  T _dt = 0;
  size_t _N_TIMESTEPS = 0;
  T _V = 0;   // actual cost of this phase only
  T _dV = 0;  // expected cost change of this phase
  size_t _xsize = 0, _usize = 4, _ysize = 4;

  size_t get_modeidx() const { return _modeidx; }
  // ModelState<T, _xsize, 4, 4>[_N_TIMESTEPS] (cast as the reference's solve_mhpc does)
  void* get_nominal_ms_ptr() { fetch(); return ms_.data(); }
  // CostToGoStruct<T, _xsize, 4>[_N_TIMESTEPS]
  void* get_CTG_info_ptr() { fetch(); return ctg_.data(); }
  std::vector<T> get_terminal_state() {
    fetch();
    const T* xN = ms_.data() + (_N_TIMESTEPS - 1) * ms_stride();
    return std::vector<T>(xN, xN + _xsize);
  }

 private:
  template <typename>
  friend class MHPCLocomotion;
  size_t ms_stride() const {
    return _xsize == 14 ? sizeof(ModelState<T, 14, 4, 4>) / sizeof(T)
                        : sizeof(ModelState<T, 6, 4, 4>) / sizeof(T);
  }
  size_t ctg_stride() const {
    return _xsize == 14 ? sizeof(CostToGoStruct<T, 14, 4>) / sizeof(T)
                        : sizeof(CostToGoStruct<T, 6, 4>) / sizeof(T);
  }
  void fetch() {
    if (!stale_) return;
    const size_t n = _xsize, N = _N_TIMESTEPS;
    std::vector<double> x(N * n), u(N * 4), y(N * 4), K(N * 4 * n), du(N * 4), G(N * n);
    const int rc = mhpc_get_phase_problems(h_, phase_, problem_, 1, x.data(), u.data(), y.data(),
                                           K.data(), du.data(), G.data());
    if (rc != MHPC_OK)
      throw std::runtime_error(std::string("mhpc_get_phase_problems: ") + mhpc_last_error());
    const size_t ms = ms_stride(), cs = ctg_stride();
    ms_.assign(N * ms, T(0));
    ctg_.assign(N * cs, T(0));
    for (size_t k = 0; k < N; ++k) {
      T* m = &ms_[k * ms];  // x, u, y contiguous (ModelState's member order)
      for (size_t i = 0; i < n; ++i) m[i] = (T)x[k * n + i];
      for (size_t i = 0; i < 4; ++i) m[n + i] = (T)u[k * 4 + i];
      for (size_t i = 0; i < 4; ++i) m[n + 4 + i] = (T)y[k * 4 + i];
      T* c = &ctg_[k * cs];  // G, du, K (column-major 4 x n)
      for (size_t i = 0; i < n; ++i) c[i] = (T)G[k * n + i];
      for (size_t i = 0; i < 4; ++i) c[n + i] = (T)du[k * 4 + i];
      for (size_t r = 0; r < 4; ++r)
        for (size_t j = 0; j < n; ++j) c[n + 4 + j * 4 + r] = (T)K[(k * 4 + r) * n + j];
    }
    stale_ = false;
  }
  mhpc_handle* h_ = nullptr;
  int phase_ = 0, problem_ = 0;
  bool stale_ = true;
  std::vector<T> ms_, ctg_;
};

template <typename TH>
class MHPCLocomotion {
 public:
  // MHPCLocomotion(MHPCUserParameters*, Gait*, HSDDP_OPTION<TH>)  (MHPCLocomotion.cpp:8-43)
  MHPCLocomotion(MHPCUserParameters* params, Gait* gait, HSDDP_OPTION<TH> option, int batch = 1,
                 int device = 0)
      : batch_(batch) {
    static_assert(sizeof(TH) == 8, "only the double instantiation exists (as in the reference)");
    const int np = params->n_wbphase + params->n_fbphase;
    desc_ = build_desc(params, gait);
    opt_ = mhpc_hsddp_option{option.alpha, option.gamma, option.update_penalty,
                             option.update_relax, option.update_regularization,
                             option.update_ReB, option.max_DDP_iter, option.max_AL_iter,
                             option.DDP_thresh, option.AL_thresh, option.AL_active,
                             option.ReB_active, option.smooth_active, 0};
    check(mhpc_create(&desc_, &opt_, batch_, device, &h_), "mhpc_create");
    _option = option;
    _n_phases = np;
    gait_ = gait->to_c();
    // default initial condition (MHPCLocomotion.cpp:37-39), projected if phase 0 is SRB
    const double x0[14] = {0.0927, -0.1093, -0.1542, 1.0957, -2.2033, 0.9742, -1.7098,
                           0.9011, 0.2756,  0.7333,  0.0446, 0.0009,  1.3219, 2.7346};
    xw_ = desc_.n_wb > 0 ? 14 : 6;
    pmax_ = np;
    refresh_phases(false);
    default_x0();
  }
  ~MHPCLocomotion() { mhpc_destroy(h_); }
  // the phase layout MHPCLocomotion::build_problem makes (MHPCLocomotion.cpp:63-104) for the
  // controller's parameters and gait at its current mode params->cmode
  static mhpc_problem_desc build_desc(const MHPCUserParameters* params, Gait* gait) {
    const int np = params->n_wbphase + params->n_fbphase;
    mhpc_problem_desc d{};
    d.n_wb = params->n_wbphase;
    d.n_fb = params->n_fbphase;
    d.dt_wb = (double)params->dt_wb;
    d.dt_fb = (double)params->dt_fb;
    d.vel_cmd = params->usrcmd ? params->usrcmd->vel : 0.f;
    d.height_cmd = params->usrcmd ? params->usrcmd->height : 0.f;
    d.precision = 64;
    const std::vector<int> seq = gait->get_mode_seq(params->cmode, np);
    const std::vector<float> tim = gait->get_timings(seq);
    for (int p = 0; p < np && p < MHPC_MAX_PHASES; ++p) {
      d.mode_seq[p] = seq[p];
      // float timing / (double)(float dt), as the reference's DVec<float> / double member
      d.N[p] = (int)std::round((double)tim[p] / (p < d.n_wb ? d.dt_wb : d.dt_fb));
    }
    return d;
  }
  MHPCLocomotion(const MHPCLocomotion&) = delete;
  MHPCLocomotion& operator=(const MHPCLocomotion&) = delete;

  // extension: per-problem initial states [batch][x0_width()] (14 when any problem has a
  // whole-body phase -- an SRB-only problem reads the first 6 of its row -- else 6)
  void set_initial_conditions(const std::vector<double>& x0) { x0_ = x0; }
  int x0_width() const { return xw_; }
  // MultiPhaseDDP::set_initial_condition for every problem of the batch (same state)
  void set_initial_condition(const std::vector<double>& x0) {
    for (int b = 0; b < batch_; ++b)
      for (int i = 0; i < xw_; ++i) x0_[(size_t)b * xw_ + i] = x0[i];
  }

  // MHPCLocomotion::update_problem (MHPCLocomotion.cpp:107-158): gait advances one mode,
  // phase buffers rotate (warm start), references follow the current initial condition
  void update_problem() {
    check(mhpc_set_x0(h_, x0_.data()), "mhpc_set_x0");
    check(mhpc_update_problem(h_, &gait_), "mhpc_update_problem");
    refresh_descs();
  }

  // extension: per-problem phase layouts in one batch -- one MHPCLocomotion per controller
  // in the reference, each built from its own Gait / gait point (MHPCLocomotion.cpp:63-104).
  // Problem b gets descs[layout_of_problem[b]] (descs[b % n] for an empty vector); the
  // initial states return to the default, initialization() precedes the next solve.
  void set_layouts(const std::vector<mhpc_problem_desc>& descs,
                   const std::vector<int32_t>& layout_of_problem = {}) {
    check(mhpc_set_layouts(h_, (int)descs.size(), descs.data(),
                           layout_of_problem.empty() ? nullptr : layout_of_problem.data()),
          "mhpc_set_layouts");
    refresh_descs();
    default_x0();
  }
  // extension: update_problem per controller -- problem b takes steps[b] gait steps of
  // gaits[gait_of_problem[b]] (0: keeps its layout and warm start); empty vectors: gaits[0]
  // for every problem, one step each
  void update_problems(const std::vector<Gait*>& gaits,
                       const std::vector<int32_t>& gait_of_problem = {},
                       const std::vector<int32_t>& steps = {}) {
    std::vector<mhpc_gait> gs;
    for (Gait* g : gaits) gs.push_back(g->to_c());
    check(mhpc_set_x0(h_, x0_.data()), "mhpc_set_x0");
    check(mhpc_update_problems(h_, (int)gs.size(), gs.data(),
                               gait_of_problem.empty() ? nullptr : gait_of_problem.data(),
                               steps.empty() ? nullptr : steps.data()),
          "mhpc_update_problems");
    refresh_descs();
  }
  mhpc_problem_desc problem_desc(int b) {
    mhpc_problem_desc d{};
    check(mhpc_get_problem_desc(h_, b, &d), "mhpc_get_problem_desc");
    return d;
  }
  int num_layouts() {
    int n = 0;
    check(mhpc_num_layouts(h_, &n), "mhpc_num_layouts");
    return n;
  }

  // execution horizon of solve_mhpc (ms_exec / CTG_exec, MHPCLocomotion.cpp:176-194): nominal
  // x [batch][Ne][14], u [batch][Ne][4], K [batch][Ne][4*14], du, G of phase 0 followed by
  // phase 1 when there are two or more WB phases (Ne = N0 (+ N1))
  struct ExecHorizon { int Ne = 0; std::vector<double> x, u, y, K, du, G; };
  ExecHorizon get_exec() {
    ExecHorizon e;
    const int np = desc_.n_wb > 1 ? 2 : 1;
    std::vector<int> Ns(np);
    for (int p = 0; p < np; ++p) Ns[p] = desc_.N[p];
    for (int p = 0; p < np; ++p) e.Ne += Ns[p];
    const size_t B = batch_, Ne = e.Ne;
    e.x.resize(B * Ne * 14); e.u.resize(B * Ne * 4); e.y.resize(B * Ne * 4);
    e.K.resize(B * Ne * 56); e.du.resize(B * Ne * 4); e.G.resize(B * Ne * 14);
    size_t off = 0;
    for (int p = 0; p < np; ++p) {
      const size_t N = Ns[p];
      std::vector<double> x(B * N * 14), u(B * N * 4), y(B * N * 4), K(B * N * 56), du(B * N * 4),
          G(B * N * 14);
      check(mhpc_get_phase(h_, p, x.data(), u.data(), y.data(), K.data(), du.data(), G.data()),
            "mhpc_get_phase");
      for (size_t b = 0; b < B; ++b) {
        auto cp = [&](std::vector<double>& dst, const std::vector<double>& src, size_t w) {
          std::copy(src.begin() + b * N * w, src.begin() + (b + 1) * N * w,
                    dst.begin() + (b * Ne + off) * w);
        };
        cp(e.x, x, 14); cp(e.u, u, 4); cp(e.y, y, 4); cp(e.K, K, 56); cp(e.du, du, 4); cp(e.G, G, 14);
      }
      off += N;
    }
    return e;
  }

  void initialization() {  // (:47-53)
    check(mhpc_set_x0(h_, x0_.data()), "mhpc_set_x0");
    check(mhpc_initialize(h_), "mhpc_initialize");
    refresh_phases(false);
  }

  void solve_mhpc() {  // (:167-195)
    status_.assign(batch_, 0);
    check(mhpc_solve(h_, status_.data()), "mhpc_solve");
    refresh_phases(true);
  }

  // extension: which problem of the batch _phases, _actual_cost, _exp_cost_change and
  // _tconstr_violation describe (default 0; the reference holds exactly one problem)
  void select_problem(int b) {
    if (b < 0 || b >= batch_) throw std::runtime_error("select_problem: no such problem");
    problem_ = b;
    if (!pdesc_.empty()) desc_ = pdesc_[b];
    refresh_phases(solved_);
  }

  // MHPCLocomotion::print_debugInfo (MHPCLocomotion.cpp:293-380) for one problem:
  // state.txt, control.txt, gradient.txt, cost.txt in Eigen's default row format, with the
  // reference's row counts -- including its N_TIMESTEPS[i+2] for the SRB phases of
  // control / gradient / cost (exact for n_wbphase = 2; rows past an SRB phase's own N are
  // the zero-initialised buffer; clamped where the reference would read past the array).
  void print_debugInfo(int problem = 0) {
    const mhpc_problem_desc dsc = pdesc_.empty() ? desc_ : pdesc_[problem];
    const int nwb = dsc.n_wb, nfb = dsc.n_fb, np = nwb + nfb;
    struct Part { int n, N; std::vector<double> x, u, g, lx, phix; };
    std::vector<Part> parts(np);
    for (int p = 0; p < np; ++p) {
      Part& q = parts[p];
      check(mhpc_phase_dims(&dsc, p, &q.n, &q.N), "mhpc_phase_dims");
      q.x.resize((size_t)q.N * q.n); q.u.resize((size_t)q.N * 4); q.g.resize((size_t)q.N * q.n);
      q.lx.resize((size_t)(q.N - 1) * q.n); q.phix.resize(q.n);
      check(mhpc_get_phase_problems(h_, p, problem, 1, q.x.data(), q.u.data(), nullptr, nullptr,
                                    nullptr, q.g.data()), "mhpc_get_phase_problems");
      check(mhpc_get_cost_gradients_problems(h_, p, problem, 1, q.lx.data(), q.phix.data()),
            "mhpc_get_cost_gradients_problems");
    }
    auto n_rows = [&](int i) { return i + 2 < np ? parts[i + 2].N : parts[nwb + i].N; };
    // rows k < want of a [N][w] block, zero rows past N
    auto block = [](std::ofstream& f, const std::vector<double>& a, int N, int w, int want) {
      const std::vector<double> zero(w, 0.0);
      for (int k = 0; k < want; ++k) write_row(f, k < N ? &a[(size_t)k * w] : zero.data(), w);
    };
    std::ofstream gradient_output("gradient.txt"), state_output("state.txt"),
        contrl_output("control.txt"), cost_output("cost.txt");
    std::printf("********** Write to file state.txt ************\n");
    for (int i = 0; i < nwb; ++i) block(state_output, parts[i].x, parts[i].N, 14, parts[i].N);
    for (int i = 0; i < nfb; ++i) {
      const Part& q = parts[nwb + i];
      block(state_output, q.x, q.N, 6, q.N);
    }
    std::printf("********** Write to file control.txt ************\n");
    for (int i = 0; i < nwb; ++i) block(contrl_output, parts[i].u, parts[i].N, 4, parts[i].N);
    for (int i = 0; i < nfb; ++i) block(contrl_output, parts[nwb + i].u, parts[nwb + i].N, 4, n_rows(i));
    std::printf("********** Write to file gradient.txt ************\n");
    for (int i = 0; i < nwb; ++i) block(gradient_output, parts[i].g, parts[i].N, 14, parts[i].N);
    for (int i = 0; i < nfb; ++i) block(gradient_output, parts[nwb + i].g, parts[nwb + i].N, 6, n_rows(i));
    std::printf("********** Write to file cost.txt ************\n");
    for (int i = 0; i < nwb; ++i) {
      block(cost_output, parts[i].lx, parts[i].N - 1, 14, parts[i].N - 1);
      write_row(cost_output, parts[i].phix.data(), 14);
    }
    for (int i = 0; i < nfb; ++i) {
      const Part& q = parts[nwb + i];
      block(cost_output, q.lx, q.N - 1, 6, n_rows(i) - 1);
      write_row(cost_output, q.phix.data(), 6);
    }
  }

  // extension: the weights / constraint parameters the reference's WBCost, FBCost and
  // WBConstraint objects hold (MHPCCost.cpp:24-75, MHPCConstraints.cpp:14-88), replaceable
  // here for every later solve (mhpc_set_cost_weights / mhpc_set_constraint_params)
  void set_cost_weights(const mhpc_cost_weights& w) {
    check(mhpc_set_cost_weights(h_, &w), "mhpc_set_cost_weights");
  }
  mhpc_cost_weights get_cost_weights() {
    mhpc_cost_weights w{};
    check(mhpc_get_cost_weights(h_, &w), "mhpc_get_cost_weights");
    return w;
  }
  void set_constraint_params(const mhpc_constraint_params& c) {
    check(mhpc_set_constraint_params(h_, &c), "mhpc_set_constraint_params");
  }
  mhpc_constraint_params get_constraint_params() {
    mhpc_constraint_params c{};
    check(mhpc_get_constraint_params(h_, &c), "mhpc_get_constraint_params");
    return c;
  }

  const std::vector<int32_t>& status() const { return status_; }
  const mhpc_problem_desc& desc() const { return desc_; }
  mhpc_handle* handle() { return h_; }

  TH _actual_cost = 0, _exp_cost_change = 0, _tconstr_violation = 0;
  // MultiPhaseDDP's public phase list: _phases[p]->_V, _dV, _N_TIMESTEPS, get_nominal_ms_ptr()...
  std::vector<SinglePhaseAbstract<TH>*> _phases;
  int _n_phases = 0;
  HSDDP_OPTION<TH> _option;

 private:
  // every problem's layout (kept only when they differ), the x0 row width, the widest
  // phase count (the row width of mhpc_get_scalars' per-phase arrays)
  void refresh_descs() {
    std::vector<mhpc_problem_desc> ds(batch_);
    bool mixed = false;
    for (int b = 0; b < batch_; ++b) {
      ds[b] = problem_desc(b);
      mixed = mixed || std::memcmp(&ds[b], &ds[0], sizeof(mhpc_problem_desc)) != 0;
    }
    xw_ = 6;
    for (const mhpc_problem_desc& d : ds)
      if (d.n_wb > 0) xw_ = 14;
    check(mhpc_max_phases(h_, &pmax_), "mhpc_max_phases");
    desc_ = ds[problem_];
    pdesc_ = mixed ? std::move(ds) : std::vector<mhpc_problem_desc>();
    refresh_phases(false);
  }
  // the reference's default initial condition (MHPCLocomotion.cpp:37-39), projected for a
  // batch without whole-body phases
  void default_x0() {
    const double x0[14] = {0.0927, -0.1093, -0.1542, 1.0957, -2.2033, 0.9742, -1.7098,
                           0.9011, 0.2756,  0.7333,  0.0446, 0.0009,  1.3219, 2.7346};
    const int proj[6] = {0, 1, 2, 7, 8, 9};
    x0_.resize((size_t)batch_ * xw_);
    for (int b = 0; b < batch_; ++b)
      for (int i = 0; i < xw_; ++i) x0_[(size_t)b * xw_ + i] = xw_ == 14 ? x0[i] : x0[proj[i]];
  }
  // phase configuration from the selected problem's current layout; costs from the last solve
  void refresh_phases(bool scalars) {
    const int np = desc_.n_wb + desc_.n_fb;
    while ((int)phase_store_.size() < np) phase_store_.emplace_back(new SinglePhaseAbstract<TH>());
    _phases.clear();
    for (int p = 0; p < np; ++p) _phases.push_back(phase_store_[p].get());
    _n_phases = np;
    const size_t pw = (size_t)pmax_;
    std::vector<double> J(batch_), dV(batch_), viol(batch_), Vp((size_t)batch_ * pw),
        dVp((size_t)batch_ * pw);
    if (scalars)
      check(mhpc_get_scalars(h_, J.data(), dV.data(), viol.data(), Vp.data(), dVp.data(), nullptr),
            "mhpc_get_scalars");
    solved_ = scalars;
    for (int p = 0; p < np; ++p) {
      SinglePhaseAbstract<TH>& q = *_phases[p];
      q.h_ = h_;
      q.phase_ = p;
      q.problem_ = problem_;
      q.stale_ = true;
      q._modeidx = desc_.mode_seq[p];
      q._phaseidx = p;
      q._dt = p < desc_.n_wb ? desc_.dt_wb : desc_.dt_fb;
      q._N_TIMESTEPS = desc_.N[p];
      q._xsize = p < desc_.n_wb ? 14 : 6;
      q._V = scalars ? (TH)Vp[(size_t)problem_ * pw + p] : TH(0);
      q._dV = scalars ? (TH)dVp[(size_t)problem_ * pw + p] : TH(0);
    }
    if (scalars) {
      _actual_cost = J[problem_];
      _exp_cost_change = dV[problem_];
      _tconstr_violation = viol[problem_];
    }
  }
  static void check(int rc, const char* what) {
    if (rc != MHPC_OK)
      throw std::runtime_error(std::string(what) + ": " + mhpc_last_error());
  }
  // `ostream << vec.transpose()` with Eigen's default IOFormat: every coefficient printed
  // like `ostream << double` (%g, 6 significant digits), right-aligned to the widest
  // coefficient of the row, one space between coefficients
  static void write_row(std::ofstream& f, const double* v, int n) {
    std::vector<std::string> s(n);
    size_t w = 0;
    char buf[40];
    for (int i = 0; i < n; ++i) {
      std::snprintf(buf, sizeof buf, "%g", v[i]);
      s[i] = buf;
      if (s[i].size() > w) w = s[i].size();
    }
    for (int i = 0; i < n; ++i) {
      if (i) f << ' ';
      f << std::string(w - s[i].size(), ' ') << s[i];
    }
    f << '\n';
  }

  int batch_;
  mhpc_gait gait_{};
  mhpc_problem_desc desc_;
  mhpc_hsddp_option opt_;
  mhpc_handle* h_ = nullptr;
  std::vector<double> x0_;
  std::vector<int32_t> status_;
  std::vector<std::unique_ptr<SinglePhaseAbstract<TH>>> phase_store_;
  std::vector<mhpc_problem_desc> pdesc_;  // per-problem layouts (empty: all equal desc_)
  int xw_ = 14, pmax_ = 0;
  int problem_ = 0;
  bool solved_ = false;
};
