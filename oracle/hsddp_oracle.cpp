// TEST INFRASTRUCTURE ONLY -- CPU oracle for the HSDDP solve path.
//
// A line-faithful restatement of the reference's Eigen code, without Eigen (absent from
// this image), whose model evaluations are the reference's OWN CasADi C
// kernels (oracle/_ref/libmhpc_casadi_ref.so, compiled from
// /root/reference/CasadiGen/source by oracle/Makefile) called with the semantics of
// casadi_interface (CasadiGen/source/CasadiGen.cpp:4-79).  Every function cites the
// reference lines it restates.  The product library never links or calls this file;
// only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline do.
//
// Parity notes: the reference's Eigen expression evaluation order is followed
// left-to-right (e.g. A'*H*A = (A'H)A), but Eigen's SIMD/FMA summation order is not
// reproducible without Eigen; the restatement is therefore pinned by the reference's
// CasADi kernels for all model arithmetic and is otherwise "parity unpinned" at the
// rounding level for the Eigen-implemented driver arithmetic.
#include "mhpc_oracle.h"

#include <dlfcn.h>
#include <math.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

namespace {

constexpr double PI = 3.141592653589793238;  // MHPC_CPPTypes.h:18

// ------------------------------------------------------------------------------------
// CasADi reference kernels (dlopen'ed), casadi_interface semantics.
typedef int (*casadi_fn)(const double**, double**, long long*, double*, int);
typedef const long long* (*casadi_sp)(long long);
typedef long long (*casadi_nout)(void);

struct CasadiFn {
  casadi_fn f = nullptr;
  casadi_sp sp = nullptr;
  int nout = 0;
};

struct RefLib {
  void* handle = nullptr;
  CasadiFn Dyn_FL, Dyn_BS, Dyn_FS, Dyn_FL_par, Dyn_BS_par, Dyn_FS_par;
  CasadiFn Imp_F, Imp_B, Imp_F_par, Imp_B_par, FBDynamics, FBDynamics_par;
  CasadiFn WB_FL1, WB_FL2, Jacob_F, Jacob_B;
} g_ref;

bool load_fn(CasadiFn& c, const char* name) {
  c.f = (casadi_fn)dlsym(g_ref.handle, name);
  std::string sp = std::string(name) + "_sparsity_out";
  std::string no = std::string(name) + "_n_out";
  c.sp = (casadi_sp)dlsym(g_ref.handle, sp.c_str());
  casadi_nout n = (casadi_nout)dlsym(g_ref.handle, no.c_str());
  if (!c.f || !c.sp || !n) return false;
  c.nout = (int)n();
  return true;
}

// casadi_interface (CasadiGen.cpp:4-79): evaluate into temporaries, then scatter each
// CSC output into the caller's column-major dense buffer (structural zeros untouched).
void casadi_call(const CasadiFn& c, std::initializer_list<const double*> args,
                 std::initializer_list<double*> outs) {
  const double* arg[8];
  int na = 0;
  for (auto a : args) arg[na++] = a;
  double tmp[8][256];
  double* res[8];
  for (int i = 0; i < c.nout; ++i) res[i] = tmp[i];
  c.f(arg, res, nullptr, nullptr, 0);
  int i = 0;
  for (double* RES : outs) {
    const long long* sp = c.sp(i);
    const long long nrow = sp[0], ncol = sp[1];
    const long long* colinfo = sp + 2;
    const long long* rowinfo = colinfo + ncol + 1;
    long long nz = 0;
    for (long long col = 0; col < ncol; ++col)
      while (nz < colinfo[col + 1]) {
        RES[rowinfo[nz] + nrow * col] = tmp[i][nz];
        ++nz;
      }
    ++i;
  }
}

// ------------------------------------------------------------------------------------
// Small dense helpers (row-major).
inline void mat_zero(double* a, int n) { memset(a, 0, sizeof(double) * n); }

// C = A' * B   with A (r x n), B (r x m)  -> C (n x m)
void matTmul(const double* A, const double* B, int r, int n, int m, double* C) {
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < m; ++j) {
      double s = 0.0;
      for (int k = 0; k < r; ++k) s += A[k * n + i] * B[k * m + j];
      C[i * m + j] = s;
    }
}
// C = A * B   with A (n x r), B (r x m)
void matmul(const double* A, const double* B, int n, int r, int m, double* C) {
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < m; ++j) {
      double s = 0.0;
      for (int k = 0; k < r; ++k) s += A[i * r + k] * B[k * m + j];
      C[i * m + j] = s;
    }
}

// Eigen-style 4x4 inverse by cofactors (compute_inverse_size4, generic path).
void inverse4(const double* m, double* inv) {
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
  for (int i = 0; i < 16; ++i) inv[i] = a[i] / det;
}

// Eigen::LDLT<>::compute(...).isPositive() on the lower triangle (diagonal pivoting,
// ldlt_inplace<Lower>::unblocked; sign bookkeeping starts at ZeroSign).  Returns true
// iff no strictly negative pivot was met.  (SinglePhase.cpp:202-209)
bool ldlt_is_positive(const double* Ain, int n) {
  double A[16];
  for (int i = 0; i < n * n; ++i) A[i] = Ain[i];
  enum { ZeroSign, PositiveSemiDef, NegativeSemiDef, Indefinite } sign = ZeroSign;
  double temp[4];
  for (int k = 0; k < n; ++k) {
    int big = k;
    double bigv = fabs(A[k * n + k]);
    for (int i = k + 1; i < n; ++i)
      if (fabs(A[i * n + i]) > bigv) { bigv = fabs(A[i * n + i]); big = i; }
    if (big != k) {
      for (int j = 0; j < k; ++j) std::swap(A[k * n + j], A[big * n + j]);
      for (int i = big + 1; i < n; ++i) std::swap(A[i * n + k], A[i * n + big]);
      std::swap(A[k * n + k], A[big * n + big]);
      for (int i = k + 1; i < big; ++i) {
        const double t = A[i * n + k];
        A[i * n + k] = A[big * n + i];
        A[big * n + i] = t;
      }
    }
    const int rs = n - k - 1;
    if (k > 0) {
      for (int j = 0; j < k; ++j) temp[j] = A[j * n + j] * A[k * n + j];
      double s = 0.0;
      for (int j = 0; j < k; ++j) s += A[k * n + j] * temp[j];
      A[k * n + k] -= s;
      for (int i = k + 1; i < n; ++i) {
        double t = 0.0;
        for (int j = 0; j < k; ++j) t += A[i * n + j] * temp[j];
        A[i * n + k] -= t;
      }
    }
    const double akk = A[k * n + k];
    const bool valid = fabs(akk) > 0.0;
    if (k == 0 && !valid) { sign = ZeroSign; break; }
    if (rs > 0 && valid)
      for (int i = k + 1; i < n; ++i) A[i * n + k] /= akk;
    if (sign == PositiveSemiDef) {
      if (akk < 0.0) sign = Indefinite;
    } else if (sign == NegativeSemiDef) {
      if (akk > 0.0) sign = Indefinite;
    } else if (sign == ZeroSign) {
      if (akk > 0.0) sign = PositiveSemiDef;
      else if (akk < 0.0) sign = NegativeSemiDef;
    }
  }
  return sign == PositiveSemiDef || sign == ZeroSign;
}

// ------------------------------------------------------------------------------------
// Problem data.
enum { CALC_DYN_AND_PAR = 0, CALC_PARTIALS_ONLY = 1, CALC_DYNAMICS_ONLY = 2 };  // MHPC_CPPTypes.h:6-8

struct Knot { double x[14], u[4], y[4]; };                               // ModelState
struct Par { double A[196], B[56], C[56], D[16]; };                       // DynDerivative
struct RCost { double l, lx[14], lu[4], ly[4], lxx[196], lux[56], luu[16], lyy[16]; };
struct CTG { double G[14], H[196], du[4], K[56], Qx[14], Qu[4], Qxx[196], Qux[56], Quu[16]; };
struct Ineq { double g, gx[14], gu[4], gy[4]; };  // gxx, guu, gyy are identically zero

struct Weights {  // MHPCCost.cpp:24-75 (diagonals)
  double Q[4][14], R[4][4], S[4][4], Qf[4][14];
};

Weights make_wb_weights() {
  Weights w{};
  const double q[14] = {0, 10, 5, 4, 4, 4, 4, 2, 1, .01, 6, 6, 6, 6};
  const double qf[4][14] = {{0, 20, 8, 3, 3, 3, 3, 3, 2, 0.01, 5, 5, 0.01, 0.01},
                            {0, 20, 8, 3, 3, 3, 3, 3, 2, 0.01, 5, 5, 5, 5},
                            {0, 20, 8, 3, 3, 3, 3, 3, 2, 0.01, 0.01, 0.01, 5, 5},
                            {0, 20, 8, 3, 3, 3, 3, 3, 2, 0.01, 5, 5, 5, 5}};
  const double r[4][4] = {{5, 5, 1, 1}, {1, 1, 1, 1}, {1, 1, 5, 5}, {1, 1, 1, 1}};
  // s[3] is never initialised by the reference (std::fill over [s[0], s[3]) , MHPCCost.cpp:43);
  // zero is taken here.  It only offsets the cost value of WB mode-4 phases (y = 0 in flight).
  const double s[4][4] = {{0, 0, 0.3, 0.3}, {0, 0, 0, 0}, {0.15, 0.15, 0, 0}, {0, 0, 0, 0}};
  for (int m = 0; m < 4; ++m) {
    for (int i = 0; i < 14; ++i) {
      w.Q[m][i] = 0.01 * q[i];
      w.Qf[m][i] = 100 * qf[m][i];
    }
    for (int i = 0; i < 4; ++i) {
      w.R[m][i] = 0.5 * r[m][i];
      w.S[m][i] = s[m][i];
    }
  }
  return w;
}

Weights make_fb_weights() {
  Weights w{};
  const double q[6] = {0, 10, 5, 2, 1, 0.01};
  const double qf[6] = {1, 20, 8, 3, 1, 0.01};
  const double r[4][4] = {{0, 0, 0.01, 0.01}, {0, 0, 0, 0}, {0.01, 0.01, 0, 0}, {0, 0, 0, 0}};
  for (int m = 0; m < 4; ++m) {
    for (int i = 0; i < 6; ++i) {
      w.Q[m][i] = 0.01 * q[i];
      w.Qf[m][i] = 100 * qf[i];
    }
    for (int i = 0; i < 4; ++i) {
      w.R[m][i] = r[m][i];
      w.S[m][i] = 0;
    }
  }
  return w;
}

// The solve's weights: the reference's values unless oracle_set_params replaced them (the
// counterpart of mhpc_set_cost_weights: the reference's Cost objects with other diagonals)
Weights kWB = make_wb_weights();
Weights kFB = make_fb_weights();

// Constraint parameters (MHPCConstraints.cpp:14-88; mhpc_set_constraint_params counterpart)
struct ConParams {
  double tq_lim = 33, mu = 0.5;
  double sigma[4] = {0, 5, 0, 5}, delta[4] = {0.1, 0.1, 0.1, 0.1},
         delta_min[4] = {0.01, 0.01, 0.01, 0.01}, eps_tq[4] = {0.01, 0.01, 0.01, 0.01},
         eps_grf[4] = {0.01, 0.01, 0.01, 0.01};
};
ConParams kCon;

struct Phase {
  bool wb;
  int n, mode, N;
  double dt;
  std::vector<Knot> act, nom, ref;
  std::vector<Par> par;
  std::vector<RCost> rc;
  std::vector<CTG> ctg;
  double Phi, Phix[14], Phixx[196];
  int ntc, npc;
  double h, hx[14], hxx[196];
  Ineq pc[19];
  double Bv[19], Bz[19], Bzz[19];
  // AL_REB_PARAMETER (MHPC_CompoundTypes.h:214-235) copied from WBConstraint params
  bool al_empty, reb_empty;
  double sigma, lambda, delta[19], delta_min[19], eps_reb[19];
  double V, dV, dVnext, Gnext[14], Hnext[196], x0[14];
};

struct Problem {
  const mhpc_problem_desc* d;
  mhpc_hsddp_option opt;  // MultiPhaseDDP::_option (phases point at it)
  std::vector<Phase> ph;
  double x0[14];
  double actual_cost = 0, exp_cost_change = 0, tconstr_violation = 0;
  double foothold[4] = {0, 0, 0, 0};  // PlanarFloatingBase::_foothold (shared scratch)
  int status = 0;
  int32_t trace[MHPC_TRACE_LEN];
  int ntrace = 0;
  int64_t cnt[6] = {0, 0, 0, 0, 0, 0};
};

// ---- models (PlanarQuadruped.cpp, PlanarFloatingBase.cpp) ---------------------------
void wb_dynamics(const double* x, const double* u, double* xn, double* y, int mode, double dt) {
  double xdot[14] = {0};
  const CasadiFn* f = mode == 1 ? &g_ref.Dyn_BS : mode == 3 ? &g_ref.Dyn_FS : &g_ref.Dyn_FL;
  casadi_call(*f, {x, u}, {xdot, y});
  for (int i = 0; i < 14; ++i) xn[i] = x[i] + xdot[i] * dt;  // PlanarQuadruped.cpp:25
}

void wb_dynamics_par(const double* x, const double* u, Par& p, int mode, double dt) {
  double Ac[196] = {0}, Bc[56] = {0}, C[56], D[16];  // column-major scratch (_Ac, _Bc)
  // C, D: the DynDerivative's own buffers (memset at allocation); column-major view
  double Ccm[56], Dcm[16];
  for (int r = 0; r < 4; ++r) {
    for (int c = 0; c < 14; ++c) Ccm[r + 4 * c] = p.C[r * 14 + c];
    for (int c = 0; c < 4; ++c) Dcm[r + 4 * c] = p.D[r * 4 + c];
  }
  const CasadiFn* f =
      mode == 1 ? &g_ref.Dyn_BS_par : mode == 3 ? &g_ref.Dyn_FS_par : &g_ref.Dyn_FL_par;
  casadi_call(*f, {x, u}, {Ac, Bc, Ccm, Dcm});
  (void)C;
  (void)D;
  for (int i = 0; i < 14; ++i)
    for (int j = 0; j < 14; ++j) p.A[i * 14 + j] = (i == j ? 1.0 : 0.0) + Ac[i + 14 * j] * dt;
  for (int i = 0; i < 14; ++i)
    for (int j = 0; j < 4; ++j) p.B[i * 4 + j] = Bc[i + 14 * j] * dt;
  for (int r = 0; r < 4; ++r) {
    for (int c = 0; c < 14; ++c) p.C[r * 14 + c] = Ccm[r + 4 * c];
    for (int c = 0; c < 4; ++c) p.D[r * 4 + c] = Dcm[r + 4 * c];
  }
}

void wb_resetmap(const double* x, double* xn, int mode) {  // PlanarQuadruped.cpp:58-78
  double y[4] = {0};
  if (mode == 2) casadi_call(g_ref.Imp_F, {x}, {xn, y});
  else if (mode == 4) casadi_call(g_ref.Imp_B, {x}, {xn, y});
  else memcpy(xn, x, sizeof(double) * 14);
}

void wb_resetmap_par(const double* x, double* Px, int mode) {  // row-major out
  double P[196] = {0};
  if (mode == 2 || mode == 4) {
    casadi_call(mode == 2 ? g_ref.Imp_F_par : g_ref.Imp_B_par, {x}, {P});
    for (int i = 0; i < 14; ++i)
      for (int j = 0; j < 14; ++j) Px[i * 14 + j] = P[i + 14 * j];
  } else {
    for (int i = 0; i < 196; ++i) Px[i] = 0;
    for (int i = 0; i < 14; ++i) Px[i * 14 + i] = 1.0;
  }
}

void fb_contact(int mode, double* s) {  // PlanarFloatingBase.cpp:9-23
  s[0] = mode == 3 ? 1 : 0;
  s[1] = mode == 1 ? 1 : 0;
}

void fb_dynamics(Problem& P, const double* x, const double* u, double* xn, double* y, int mode,
                 double dt) {
  double s[2], xdot[6] = {0};
  fb_contact(mode, s);
  casadi_call(g_ref.FBDynamics, {x, u, P.foothold, s}, {xdot});
  for (int i = 0; i < 4; ++i) y[i] = 0;
  for (int i = 0; i < 6; ++i) xn[i] = x[i] + xdot[i] * dt;
}

void fb_dynamics_par(Problem& P, const double* x, const double* u, Par& p, int mode, double dt) {
  double s[2], Ac[36] = {0}, Bc[24] = {0};
  fb_contact(mode, s);
  casadi_call(g_ref.FBDynamics_par, {x, u, P.foothold, s}, {Ac, Bc});
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j < 6; ++j) p.A[i * 6 + j] = (i == j ? 1.0 : 0.0) + Ac[i + 6 * j] * dt;
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j < 4; ++j) p.B[i * 4 + j] = Bc[i + 6 * j] * dt;
  mat_zero(p.C, 24);
  mat_zero(p.D, 16);
}

// FootholdPlanner::get_foothold_location (FootholdPlan.h:26-50); velcmd 1.5 and ground
// -0.404 are hard-coded by the reference (MHPCLocomotion.cpp:25).
void plan_foothold(Problem& P, const double* x0, double stance_time, int mode) {
  double f[4] = {0, 0, 0, 0};
  const double velcmd = 1.5, ground = -0.404;
  if (mode == 1) {  // back hip (H_hip): body position + R(-th) * (-0.19, 0, 0)
    const double hipx = cos(x0[2]) * (-0.19) + x0[0];
    f[2] = hipx + velcmd * stance_time / 2;
    f[3] = ground;
  } else if (mode == 3) {
    const double hipx = cos(x0[2]) * 0.19 + x0[0];
    f[0] = hipx + velcmd * stance_time / 2;
    f[1] = ground;
  }
  memcpy(P.foothold, f, sizeof f);
}

// ---- costs (CostBase.cpp:4-60) --------------------------------------------------------
void running_cost(const Phase& ph, const Knot& s, const Knot& r, RCost& rc) {
  const Weights& w = ph.wb ? kWB : kFB;
  const int m = ph.mode - 1, n = ph.n;
  double l = 0, t = 0;
  for (int i = 0; i < n; ++i) { const double d = s.x[i] - r.x[i]; l += d * w.Q[m][i] * d; }
  for (int i = 0; i < 4; ++i) { const double d = s.u[i] - r.u[i]; t += d * w.R[m][i] * d; }
  l += t;
  t = 0;
  for (int i = 0; i < 4; ++i) { const double d = s.y[i] - r.y[i]; t += d * w.S[m][i] * d; }
  l += t;
  rc.l = l * ph.dt;
}

void running_cost_par(const Phase& ph, const Knot& s, const Knot& r, RCost& rc) {
  const Weights& w = ph.wb ? kWB : kFB;
  const int m = ph.mode - 1, n = ph.n;
  const double c = 2 * ph.dt;
  mat_zero(rc.lxx, n * n);
  mat_zero(rc.lux, 4 * n);
  mat_zero(rc.luu, 16);
  mat_zero(rc.lyy, 16);
  for (int i = 0; i < n; ++i) {
    rc.lx[i] = (c * w.Q[m][i]) * (s.x[i] - r.x[i]);
    rc.lxx[i * n + i] = c * w.Q[m][i];
  }
  for (int i = 0; i < 4; ++i) {
    rc.lu[i] = (c * w.R[m][i]) * (s.u[i] - r.u[i]);
    rc.ly[i] = (c * w.S[m][i]) * (s.y[i] - r.y[i]);
    rc.luu[i * 4 + i] = c * w.R[m][i];
    rc.lyy[i * 4 + i] = c * w.S[m][i];
  }
}

void terminal_cost(Phase& ph, const Knot& s, const Knot& r) {
  const Weights& w = ph.wb ? kWB : kFB;
  const int m = ph.mode - 1;
  double l = 0;
  for (int i = 0; i < ph.n; ++i) { const double d = s.x[i] - r.x[i]; l += d * w.Qf[m][i] * d; }
  ph.Phi = l * 0.5;
}

void terminal_cost_par(Phase& ph, const Knot& s, const Knot& r) {
  const Weights& w = ph.wb ? kWB : kFB;
  const int m = ph.mode - 1, n = ph.n;
  mat_zero(ph.Phixx, n * n);
  for (int i = 0; i < n; ++i) {
    ph.Phix[i] = w.Qf[m][i] * (s.x[i] - r.x[i]);
    ph.Phixx[i * n + i] = w.Qf[m][i];
  }
}

// ---- constraints (MHPCConstraints.cpp:91-176) ------------------------------------------
const double kJointB[8] = {PI / 4, -0.1, 1.15 * PI, -0.1, PI, PI - 0.2, .1, PI - 0.2};

void path_constraint(Phase& ph, const Knot& s) {
  if (!ph.wb) return;  // FBConstraint::path_constraint is empty
  for (int i = 0; i < 8; ++i) {  // torque_limit
    Ineq& c = ph.pc[i];
    const double sgn = i < 4 ? -1.0 : 1.0;
    c.g = sgn * s.u[i % 4] + kCon.tq_lim;
    c.gu[i % 4] = sgn;
  }
  for (int i = 0; i < 8; ++i) {  // joint_limit
    Ineq& c = ph.pc[8 + i];
    const double sgn = i < 4 ? -1.0 : 1.0;
    c.g = sgn * s.x[3 + i % 4] + kJointB[i];
    c.gx[3 + i % 4] = sgn;
  }
  if (ph.mode == 1 || ph.mode == 3) {  // GRF_constraint
    const double mu = kCon.mu;
    const int o = ph.mode == 1 ? 2 : 0;  // back foot force in y[2:4], front in y[0:2]
    double rows[3][4] = {{0}};
    rows[0][o + 1] = 1;
    rows[1][o] = -1; rows[1][o + 1] = mu;
    rows[2][o] = 1;  rows[2][o + 1] = mu;
    for (int i = 0; i < 3; ++i) {
      Ineq& c = ph.pc[16 + i];
      double g = 0;
      for (int j = 0; j < 4; ++j) g += rows[i][j] * s.y[j];
      c.g = g + 0;
      for (int j = 0; j < 4; ++j) c.gy[j] = rows[i][j];
    }
  }
}

void terminal_constraint(Phase& ph, const Knot& s) {
  if (!ph.wb || ph.ntc == 0) return;
  double hx[14] = {0}, hxx[196] = {0}, hxxcm[196] = {0};
  double h = 0;
  casadi_call(ph.mode == 2 ? g_ref.WB_FL1 : g_ref.WB_FL2, {s.x}, {&h, hx, hxxcm});
  ph.h = h;
  memcpy(ph.hx, hx, sizeof hx);
  for (int i = 0; i < 14; ++i)
    for (int j = 0; j < 14; ++j) hxx[i * 14 + j] = hxxcm[i + 14 * j];
  memcpy(ph.hxx, hxx, sizeof hxx);
}

// SinglePhase::reduced_barrier (SinglePhase.cpp:298-317)
void reduced_barrier(Phase& ph) {
  const int k = 2;
  for (int i = 0; i < ph.npc; ++i) {
    const double g = ph.pc[i].g, dl = ph.delta[i];
    if (g > dl) {
      ph.Bv[i] = -log(g);
      ph.Bz[i] = -1.0 / g;
      ph.Bzz[i] = pow(g, -2);
    } else {
      const double t = (g - k * dl) / ((k - 1) * dl);
      ph.Bv[i] = (double)(k - 1) / k * (pow(t, k) - 1) - log(dl);
      ph.Bz[i] = pow(t, k - 1) / dl;
      ph.Bzz[i] = pow(t, k - 2);
    }
  }
}

// SinglePhase::update_running_cost_with_pconstr (SinglePhase.cpp:219-249)
void update_running_cost_with_pconstr(Phase& ph, RCost& rc, int flag) {
  for (int i = 0; i < ph.npc; ++i) { ph.Bv[i] = 0; ph.Bz[i] = 0; ph.Bzz[i] = 0; }
  reduced_barrier(ph);
  const int n = ph.n;
  for (int i = 0; i < ph.npc; ++i) {
    const double e = ph.eps_reb[i], B = ph.Bv[i], Bz = ph.Bz[i], Bzz = ph.Bzz[i];
    const Ineq& c = ph.pc[i];
    if (flag == CALC_DYNAMICS_ONLY || flag == CALC_DYN_AND_PAR) rc.l += e * B * ph.dt;
    if (flag == CALC_PARTIALS_ONLY || flag == CALC_DYN_AND_PAR) {
      for (int a = 0; a < n; ++a) rc.lx[a] += e * Bz * c.gx[a] * ph.dt;
      for (int a = 0; a < 4; ++a) rc.lu[a] += e * Bz * c.gu[a] * ph.dt;
      for (int a = 0; a < 4; ++a) rc.ly[a] += e * Bz * c.gy[a] * ph.dt;
      for (int a = 0; a < n; ++a)
        for (int b = 0; b < n; ++b) rc.lxx[a * n + b] += e * (c.gx[a] * Bzz * c.gx[b]) * ph.dt;
      for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b) rc.luu[a * 4 + b] += e * (c.gu[a] * Bzz * c.gu[b]) * ph.dt;
      for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b) rc.lyy[a * 4 + b] += e * (c.gy[a] * Bzz * c.gy[b]) * ph.dt;
    }
  }
}

// SinglePhase::update_terminal_cost_with_tconstr (SinglePhase.cpp:257-275), including the
// guard quirk of :269 (partials added in DYNAMICS_ONLY and DYN_AND_PAR, not PARTIALS_ONLY).
void update_terminal_cost_with_tconstr(Phase& ph, int flag) {
  const int n = ph.n;
  for (int idx = 0; idx < ph.ntc; ++idx) {
    const double s = ph.sigma, lam = ph.lambda, h = ph.h;
    if (flag == CALC_DYNAMICS_ONLY || flag == CALC_DYN_AND_PAR)
      ph.Phi += 50 * (pow(s * h / 2, 2) + lam * h);
    if (flag == CALC_DYNAMICS_ONLY || flag == CALC_DYN_AND_PAR) {
      for (int i = 0; i < n; ++i) ph.Phix[i] += 50 * (s * s / 2 * ph.hx[i] * h + lam * ph.hx[i]);
      for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j)
          ph.Phixx[i * n + j] += 50 * (s * s / 2 * (ph.hx[i] * ph.hx[j] + h * ph.hxx[i * n + j]) +
                                      lam * ph.hxx[i * n + j]);
    }
  }
}

void model_dynamics(Problem& P, Phase& ph, Knot& s, Knot& sn) {
  if (ph.wb) wb_dynamics(s.x, s.u, sn.x, s.y, ph.mode, ph.dt);
  else fb_dynamics(P, s.x, s.u, sn.x, s.y, ph.mode, ph.dt);
}

void model_par(Problem& P, Phase& ph, Knot& s, Par& p) {
  if (ph.wb) wb_dynamics_par(s.x, s.u, p, ph.mode, ph.dt);
  else fb_dynamics_par(P, s.x, s.u, p, ph.mode, ph.dt);
}

void control_update(const Phase& ph, int k, double eps, Knot& a) {  // SinglePhase.cpp:76
  const Knot& nm = ph.nom[k];
  const CTG& c = ph.ctg[k];
  for (int i = 0; i < 4; ++i) {
    double fb = 0;
    for (int j = 0; j < ph.n; ++j) fb += c.K[i * ph.n + j] * (a.x[j] - nm.x[j]);
    a.u[i] = nm.u[i] + eps * c.du[i] + fb;
  }
}

// SinglePhase::forward_sweep (SinglePhase.cpp:62-114)
void phase_forward_sweep(Problem& P, Phase& ph, double eps) {
  ph.V = 0;
  memcpy(ph.act[0].x, ph.x0, sizeof(double) * ph.n);
  if (!ph.wb) plan_foothold(P, ph.x0, ph.dt * ph.N, ph.mode);
  for (int k = 0; k < ph.N - 1; ++k) {
    control_update(ph, k, eps, ph.act[k]);
    model_dynamics(P, ph, ph.act[k], ph.act[k + 1]);
    model_par(P, ph, ph.act[k], ph.par[k]);
    running_cost(ph, ph.act[k], ph.ref[k], ph.rc[k]);
    running_cost_par(ph, ph.act[k], ph.ref[k], ph.rc[k]);
    path_constraint(ph, ph.act[k]);
    if (P.opt.ReB_active && !ph.reb_empty) update_running_cost_with_pconstr(ph, ph.rc[k], CALC_DYN_AND_PAR);
    ph.V += ph.rc[k].l;
  }
  const int e = ph.N - 1;
  terminal_cost(ph, ph.act[e], ph.ref[e]);
  terminal_cost_par(ph, ph.act[e], ph.ref[e]);
  terminal_constraint(ph, ph.act[e]);
  if (P.opt.AL_active & !ph.al_empty) update_terminal_cost_with_tconstr(ph, CALC_DYN_AND_PAR);
  ph.V += ph.Phi;
}

// SinglePhase::forward_sweep_dynamics_only (SinglePhase.cpp:117-144)
void phase_forward_sweep_dynamics_only(Problem& P, Phase& ph, double eps) {
  ph.V = 0;
  memcpy(ph.act[0].x, ph.x0, sizeof(double) * ph.n);
  if (!ph.wb) plan_foothold(P, ph.x0, ph.dt * ph.N, ph.mode);
  for (int k = 0; k < ph.N - 1; ++k) {
    control_update(ph, k, eps, ph.act[k]);
    model_dynamics(P, ph, ph.act[k], ph.act[k + 1]);
    running_cost(ph, ph.act[k], ph.ref[k], ph.rc[k]);
    path_constraint(ph, ph.act[k]);
    if (P.opt.ReB_active && !ph.reb_empty) update_running_cost_with_pconstr(ph, ph.rc[k], CALC_DYNAMICS_ONLY);
    ph.V += ph.rc[k].l;
  }
  const int e = ph.N - 1;
  terminal_cost(ph, ph.act[e], ph.ref[e]);
  terminal_constraint(ph, ph.act[e]);
  if (P.opt.AL_active & !ph.al_empty) update_terminal_cost_with_tconstr(ph, CALC_DYNAMICS_ONLY);
  ph.V += ph.Phi;
}

// SinglePhase::forward_sweep_partials_only (SinglePhase.cpp:147-180)
void phase_partials_only(Problem& P, Phase& ph) {
  if (!ph.wb) plan_foothold(P, ph.x0, ph.dt * ph.N, ph.mode);
  for (int k = 0; k < ph.N - 1; ++k) {
    model_par(P, ph, ph.act[k], ph.par[k]);
    running_cost_par(ph, ph.act[k], ph.ref[k], ph.rc[k]);
    path_constraint(ph, ph.act[k]);
    if (P.opt.ReB_active && !ph.reb_empty) update_running_cost_with_pconstr(ph, ph.rc[k], CALC_PARTIALS_ONLY);
  }
  const int e = ph.N - 1;
  terminal_cost_par(ph, ph.act[e], ph.ref[e]);
  terminal_constraint(ph, ph.act[e]);
  if (P.opt.AL_active & !ph.al_empty) update_terminal_cost_with_tconstr(ph, CALC_PARTIALS_ONLY);
}

// CostToGoStruct::compute_Qfunction (MHPC_CompoundTypes.h:117-126)
void compute_Qfunction(CTG& c, const RCost& rc, const Par& p, const double* Gn, const double* Hn, int n) {
  double t[196], t2[196], AtH[196], BtH[56], Ctl[56], Dtl[16];
  // Qx = lx + A'G + C'ly
  matTmul(p.A, Gn, n, n, 1, t);
  matTmul(p.C, rc.ly, 4, n, 1, t2);
  for (int i = 0; i < n; ++i) c.Qx[i] = rc.lx[i] + t[i] + t2[i];
  matTmul(p.B, Gn, n, 4, 1, t);
  matTmul(p.D, rc.ly, 4, 4, 1, t2);
  for (int i = 0; i < 4; ++i) c.Qu[i] = rc.lu[i] + t[i] + t2[i];
  // Qxx = lxx + (C'lyy)C + (A'H)A
  matTmul(p.C, rc.lyy, 4, n, 4, Ctl);
  matmul(Ctl, p.C, n, 4, n, t);
  matTmul(p.A, Hn, n, n, n, AtH);
  matmul(AtH, p.A, n, n, n, t2);
  for (int i = 0; i < n * n; ++i) c.Qxx[i] = rc.lxx[i] + t[i] + t2[i];
  // Quu = luu + (D'lyy)D + (B'H)B
  matTmul(p.D, rc.lyy, 4, 4, 4, Dtl);
  matmul(Dtl, p.D, 4, 4, 4, t);
  matTmul(p.B, Hn, n, 4, n, BtH);
  matmul(BtH, p.B, 4, n, 4, t2);
  for (int i = 0; i < 16; ++i) c.Quu[i] = rc.luu[i] + t[i] + t2[i];
  // Qux = lux + (D'lyy)C + (B'H)A
  matmul(Dtl, p.C, 4, 4, n, t);
  matmul(BtH, p.A, 4, n, n, t2);
  for (int i = 0; i < 4 * n; ++i) c.Qux[i] = rc.lux[i] + t[i] + t2[i];
}

// CostToGoStruct::valuefunction_update (MHPC_CompoundTypes.h:128-144)
double valuefunction_update(CTG& c, int n) {
  double inv[16], Qi[16], t[56], w[196];
  inverse4(c.Quu, inv);
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) Qi[i * 4 + j] = (inv[i * 4 + j] + inv[j * 4 + i]) / 2;
  double Qs[196];
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) Qs[i * n + j] = (c.Qxx[i * n + j] + c.Qxx[j * n + i]) / 2;
  memcpy(c.Qxx, Qs, sizeof(double) * n * n);
  for (int i = 0; i < 4; ++i) {
    double s = 0;
    for (int j = 0; j < 4; ++j) s += -Qi[i * 4 + j] * c.Qu[j];
    c.du[i] = s;
  }
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < n; ++j) {
      double s = 0;
      for (int k = 0; k < 4; ++k) s += -Qi[i * 4 + k] * c.Qux[k * n + j];
      c.K[i * n + j] = s;
    }
  matTmul(c.Qux, Qi, 4, n, 4, t);  // Qux' * Quu_inv  (n x 4)
  for (int i = 0; i < n; ++i) {
    double s = 0;
    for (int k = 0; k < 4; ++k) s += t[i * 4 + k] * c.Qu[k];
    c.G[i] = c.Qx[i] - s;
  }
  matmul(t, c.Qux, n, 4, n, w);
  for (int i = 0; i < n * n; ++i) c.H[i] = c.Qxx[i] - w[i];
  double r[4];
  for (int j = 0; j < 4; ++j) {  // Qu' * Quu^-1
    double s = 0;
    for (int k = 0; k < 4; ++k) s += c.Qu[k] * inv[k * 4 + j];
    r[j] = s;
  }
  double dV = 0;
  for (int j = 0; j < 4; ++j) dV += r[j] * c.Qu[j];
  return -dV;
}

// SinglePhase::backward_sweep (SinglePhase.cpp:183-216)
bool phase_backward_sweep(Problem& P, Phase& ph, double reg) {
  const int n = ph.n;
  ph.dV = ph.dVnext;
  CTG& last = ph.ctg[ph.N - 1];
  for (int i = 0; i < n; ++i) last.G[i] = ph.Phix[i] + ph.Gnext[i];
  for (int i = 0; i < n * n; ++i) last.H[i] = ph.Phixx[i] + ph.Hnext[i];
  const double eps9 = pow(0.1, 9);
  for (int k = ph.N - 2; k >= 0; --k) {
    CTG& c = ph.ctg[k];
    compute_Qfunction(c, ph.rc[k], ph.par[k], ph.ctg[k + 1].G, ph.ctg[k + 1].H, n);
    for (int i = 0; i < n; ++i) c.Qxx[i * n + i] += 1.0 * reg;
    for (int i = 0; i < 4; ++i) c.Quu[i * 4 + i] += 1.0 * reg;
    P.cnt[2]++;
    double Qr[16];
    for (int i = 0; i < 16; ++i) Qr[i] = c.Quu[i] - ((i % 5 == 0) ? 1.0 * eps9 : 0.0);
    if (!ldlt_is_positive(Qr, 4)) return false;
    ph.dV += valuefunction_update(c, n);
  }
  return true;
}

// ---- MultiPhaseDDP (MultiPhaseDDP.cpp) -------------------------------------------------
const double kProj[6] = {0, 1, 2, 7, 8, 9};  // rows of _stateProj (MHPCLocomotion.cpp:32-34)

// MultiPhaseDDP::phase_transition (:351-379)
void phase_transition(Problem& P, int p, double* x0next) {
  Phase& c = P.ph[p];
  Phase& nx = P.ph[p + 1];
  const double* xe = c.act[c.N - 1].x;
  if (c.wb) {
    double xi[14] = {0};
    wb_resetmap(xe, xi, c.mode);
    if (nx.wb) memcpy(x0next, xi, sizeof xi);
    else for (int i = 0; i < 6; ++i) x0next[i] = xi[(int)kProj[i]];
  } else {
    memcpy(x0next, xe, sizeof(double) * c.n);
  }
}

void mp_forward_sweep(Problem& P, double eps, bool dyn_only) {
  P.actual_cost = 0;
  double x0[14];
  memcpy(x0, P.x0, sizeof x0);
  P.tconstr_violation = 0;
  const int np = (int)P.ph.size();
  for (int p = 0; p < np; ++p) {
    memcpy(P.ph[p].x0, x0, sizeof(double) * P.ph[p].n);
    if (dyn_only) phase_forward_sweep_dynamics_only(P, P.ph[p], eps);
    else phase_forward_sweep(P, P.ph[p], eps);
    if (p + 1 < np) phase_transition(P, p, x0);
    P.actual_cost += P.ph[p].V;
    P.tconstr_violation += P.ph[p].ntc ? P.ph[p].h * P.ph[p].h : 0.0;
  }
  P.tconstr_violation = sqrt(P.tconstr_violation);
}

// MultiPhaseDDP::impact_aware_step (:300-341)
void impact_aware_step(Problem& P, int p, double& dV, double* G, double* H) {
  Phase& c = P.ph[p];
  Phase& nx = P.ph[p + 1];
  const int m = nx.n;
  dV = nx.dV;
  const double* Gp = nx.ctg[0].G;
  const double* Hp = nx.ctg[0].H;
  if (c.wb) {
    double Px[196];
    wb_resetmap_par(c.act[c.N - 1].x, Px, c.mode);
    if (nx.wb) {
      matTmul(Px, Gp, 14, 14, 1, G);
      double t[196];
      matTmul(Px, Hp, 14, 14, 14, t);
      matmul(t, Px, 14, 14, 14, H);
    } else {
      double PT[14 * 6];  // Px' * P'  (14 x 6)
      for (int i = 0; i < 14; ++i)
        for (int j = 0; j < 6; ++j) PT[i * 6 + j] = Px[(int)kProj[j] * 14 + i];
      matmul(PT, Gp, 14, 6, 1, G);
      double t1[14 * 6], t2[196];
      matmul(PT, Hp, 14, 6, 6, t1);
      // (. * P): 14x6 times 6x14 selector
      for (int i = 0; i < 14; ++i)
        for (int j = 0; j < 14; ++j) t2[i * 14 + j] = 0;
      for (int i = 0; i < 14; ++i)
        for (int j = 0; j < 6; ++j) t2[i * 14 + (int)kProj[j]] = t1[i * 6 + j];
      matmul(t2, Px, 14, 14, 14, H);
    }
  } else {
    memcpy(G, Gp, sizeof(double) * m);
    memcpy(H, Hp, sizeof(double) * m * m);
  }
}

bool mp_backward_sweep(Problem& P, double reg) {
  const int np = (int)P.ph.size();
  double dVnext = 0, G[14] = {0}, H[196] = {0};
  bool ok = true;
  P.cnt[1]++;
  for (int p = np - 1; p >= 0; --p) {
    if (p + 1 < np) impact_aware_step(P, p, dVnext, G, H);
    Phase& ph = P.ph[p];
    ph.dVnext = dVnext;
    memcpy(ph.Gnext, G, sizeof(double) * ph.n);
    memcpy(ph.Hnext, H, sizeof(double) * ph.n * ph.n);
    if (!phase_backward_sweep(P, ph, reg)) { ok = false; break; }
  }
  if (ok) P.exp_cost_change = P.ph[0].dV;
  return ok;
}

int mp_forward_iteration(Problem& P) {  // :130-151
  double eps = 1;
  const double cost_prev = P.actual_cost;
  int iter = 1;
  while (eps > pow(0.1, 10)) {
    mp_forward_sweep(P, eps, true);
    P.cnt[3]++;
    if (P.actual_cost <= cost_prev + P.opt.gamma * eps * (1 - eps / 2) * P.exp_cost_change) break;
    eps *= P.opt.alpha;
    iter++;
  }
  return iter;
}

void update_nominal(Problem& P) {
  for (auto& ph : P.ph) ph.nom = ph.act;  // memcpy of all N knots (SinglePhase.cpp:358-361)
}

void update_AL_ReB_param(Problem& P) {  // SinglePhase.cpp:334-354
  for (auto& ph : P.ph) {
    if (ph.ntc) ph.lambda += ph.sigma * ph.h;
    ph.sigma *= P.opt.update_penalty;
    if (P.opt.ReB_active) {
      for (int i = 0; i < ph.npc; ++i) {
        ph.delta[i] *= P.opt.update_relax;
        if (ph.delta[i] < ph.delta_min[i]) ph.delta[i] = ph.delta_min[i];
        ph.eps_reb[i] *= P.opt.update_ReB;
      }
    }
  }
}

void push_trace(Problem& P, int al, int reb, int conv, int abort_, int nls, int nbws) {
  if (P.ntrace >= MHPC_TRACE_LEN) return;
  P.trace[P.ntrace++] = (al << 24) | (reb << 23) | (conv << 22) | (abort_ << 21) |
                        ((nls & 0xff) << 8) | (nbws & 0xff);
}

// MultiPhaseDDP::solve (:154-289)
void mp_solve(Problem& P) {
  int iter_AL = 1;
  const double update_penalty = P.opt.update_penalty;
  const bool ReB_active = P.opt.ReB_active;
  while (iter_AL <= P.opt.max_AL_iter) {
    P.opt.ReB_active = ReB_active;
    if ((P.tconstr_violation > 0.05) || 1 == iter_AL) P.opt.ReB_active = 0;
    mp_forward_sweep(P, 0, false);
    P.cnt[4]++;
    update_nominal(P);
    int iter_DDP = 1;
    double reg = 0;
    while (iter_DDP <= P.opt.max_DDP_iter) {
      const double cost_prev = P.actual_cost;
      bool ok = false;
      int bws_iter = 1;
      P.cnt[0]++;
      while (!ok) {
        ok = mp_backward_sweep(P, reg);
        if (ok) break;
        reg = std::max(reg * P.opt.update_regularization, 1e-03);
        bws_iter++;
        if (reg > 1000) {
          push_trace(P, iter_AL, P.opt.ReB_active, 0, 1, 0, bws_iter);
          P.status = MHPC_SOLVE_REG_ABORT;
          return;
        }
      }
      reg = reg / 20;
      if (reg < 1e-06) reg = 0;
      const int nls = mp_forward_iteration(P);
      update_nominal(P);
      const bool conv = cost_prev - P.actual_cost < P.opt.DDP_thresh;
      push_trace(P, iter_AL, P.opt.ReB_active, conv, 0, nls, bws_iter);
      if (conv) break;
      for (auto& ph : P.ph) phase_partials_only(P, ph);
      P.cnt[5]++;
      iter_DDP++;
    }
    P.opt.update_penalty = update_penalty;
    if (P.tconstr_violation < 0.03) P.opt.update_penalty = 0;
    update_AL_ReB_param(P);
    if (P.tconstr_violation < P.opt.AL_thresh) break;
    iter_AL++;
  }
  // the boundary's status extension (include/mhpc_capi.h; the reference returns nothing):
  // a solve that ran to the end with a non-finite total cost
  if (P.status == MHPC_SOLVE_OK && !std::isfinite(P.actual_cost)) P.status = MHPC_SOLVE_NONFINITE;
}

// ---- problem construction (MHPCLocomotion::build_problem, ReferenceGen, warmstart) -----
void init_params(Phase& ph) {  // WBConstraint ctor / initialize_AL_REB_PARAMS (:14-88)
  ph.al_empty = true;
  ph.reb_empty = true;
  ph.sigma = 0;
  ph.lambda = 0;
  ph.ntc = 0;
  ph.npc = 0;
  if (!ph.wb) return;
  const int m = ph.mode;
  ph.npc = (m == 1 || m == 3) ? 19 : 16;
  ph.ntc = (m == 2 || m == 4) ? 1 : 0;
  for (int i = 0; i < ph.npc; ++i) {
    ph.delta[i] = kCon.delta[m - 1];
    ph.delta_min[i] = kCon.delta_min[m - 1];
    // torque limits 0..7, joint limits 8..15 (eps_ReB 0), GRF 16..18
    ph.eps_reb[i] = i < 8 ? kCon.eps_tq[m - 1] : i < 16 ? 0.0 : kCon.eps_grf[m - 1];
  }
  ph.reb_empty = false;
  if (m == 2 || m == 4) {
    ph.sigma = kCon.sigma[m - 1];
    ph.al_empty = false;
  }
}

void generate_ref(Problem& P) {  // ReferenceGen.{h:53-109, cpp:23-66}
  const mhpc_problem_desc& d = *P.d;
  const int np = (int)P.ph.size();
  const double vel = d.vel_cmd, hgt = d.height_cmd, GRF = 8.252 * 9.81;
  double term[4][14] = {
      {0, -0.1432, -PI / 25, 0.35 * PI, -0.65 * PI, 0.35 * PI, -0.6 * PI, vel, 1, 0, 0, 0, 0, 0},
      {0, -0.1418, PI / 35, 0.2 * PI, -0.58 * PI, 0.25 * PI, -0.7 * PI, vel, -1, 0, 0, 0, 0, 0},
      {0, -0.1325, -PI / 40, 0.33 * PI, -0.48 * PI, 0.33 * PI, -0.75 * PI, vel, 1, 0, 0, 0, 0, 0},
      {0, -0.1490, -PI / 25, 0.35 * PI, -0.7 * PI, 0.25 * PI, -0.60 * PI, vel, -1, 0, 0, 0, 0, 0}};
  const double qb[4] = {0.3 * PI, -0.7 * PI, 0.3 * PI, -0.7 * PI};
  std::vector<std::vector<double>> pos(np);
  for (int p = 0; p < np; ++p) {
    const double dt = P.ph[p].wb ? d.dt_wb : d.dt_fb;
    pos[p].resize(P.ph[p].N);
    pos[p][0] = p == 0 ? P.x0[0] : pos[p - 1][P.ph[p - 1].N - 1];
    for (int k = 1; k < P.ph[p].N; ++k) pos[p][k] = pos[p][k - 1] + vel * dt;
  }
  for (int p = 0; p < np; ++p) {
    Phase& ph = P.ph[p];
    for (int k = 0; k < ph.N - 1; ++k) {
      Knot& r = ph.ref[k];
      if (ph.wb) {
        const double xr[14] = {pos[p][k], hgt, 0, qb[0], qb[1], qb[2], qb[3], vel, 0, 0, 0, 0, 0, 0};
        memcpy(r.x, xr, sizeof xr);
        const double yr[4] = {0, GRF, 0, GRF};
        memcpy(r.y, yr, sizeof yr);
      } else {
        const double xr[6] = {pos[p][k], hgt, 0, vel, 0, 0};
        memcpy(r.x, xr, sizeof xr);
        const double ur[4] = {0, GRF, 0, GRF};
        memcpy(r.u, ur, sizeof ur);
      }
    }
    Knot& r = ph.ref[ph.N - 1];
    if (ph.wb) {
      memcpy(r.x, term[ph.mode - 1], sizeof(double) * 14);
      r.x[0] = pos[p][ph.N - 1];
    } else {
      const double t5[5] = {hgt, 0, vel, 0, 0};
      memcpy(r.x + 1, t5, sizeof t5);
      r.x[0] = pos[p][ph.N - 1];
    }
  }
}

// bounding_PDcontrol (boundingPDControl.cpp:3-46)
void bounding_pd(Phase& ph) {
  const double qnom[4] = {PI / 4, -PI * 7 / 12, PI / 4, -PI * 7 / 12};
  const double legext_nom = 0.2462, Kspring = 2200;
  const double Kp[4] = {5 * 8.0, 5 * 1.0, 5 * 12.0, 5 * 10.0};
  for (int k = 0; k < ph.N - 1; ++k) {
    Knot& s = ph.act[k];
    const int m = ph.mode;
    if (m == 1 || m == 3) {
      const int foot = m == 1 ? 1 : 0;
      double J[14] = {0}, Jd[14] = {0};  // column-major 2x7
      casadi_call(foot == 0 ? g_ref.Jacob_F : g_ref.Jacob_B, {s.x}, {J, Jd});
      // leg extension vector: foot - hip (get_leg_ext_vec via homogeneous transforms)
      const double* q = s.x;
      const int ih = 3 + 2 * foot, ik = ih + 1;
      const double a1 = q[2] + q[ih], a2 = a1 + q[ik];
      const double v0 = -0.209 * sin(a1) - 0.195 * sin(a2);
      const double v1 = -0.209 * cos(a1) - 0.195 * cos(a2);
      const double sq = v0 * v0 + v1 * v1, nrm = sqrt(sq);
      const double n0 = v0 / nrm, n1 = v1 / nrm;
      const double F0 = -n0 * Kspring * (nrm - legext_nom);
      const double F1 = -n1 * Kspring * (nrm - legext_nom);
      const double gain = m == 1 ? 3 : 2.2;
      for (int i = 0; i < 4; ++i) {
        const int col = 3 + i;
        s.u[i] = (J[0 + 2 * col] * F0 + J[1 + 2 * col] * F1) * gain;
      }
    } else {
      for (int i = 0; i < 4; ++i) s.u[i] = Kp[i] * (qnom[i] - s.x[3 + i]) - s.x[10 + i];
    }
    wb_dynamics(s.x, s.u, ph.act[k + 1].x, s.y, m, ph.dt);
  }
}

void build(Problem& P, const mhpc_problem_desc* d, const mhpc_hsddp_option* o, const double* x0) {
  P.d = d;
  P.opt = *o;
  const int np = d->n_wb + d->n_fb;
  P.ph.resize(np);
  for (int p = 0; p < np; ++p) {
    Phase& ph = P.ph[p];
    ph.wb = p < d->n_wb;
    ph.n = ph.wb ? 14 : 6;
    ph.mode = d->mode_seq[p];
    ph.N = d->N[p];
    ph.dt = ph.wb ? d->dt_wb : d->dt_fb;
    ph.act.assign(ph.N, Knot{});
    ph.nom.assign(ph.N, Knot{});
    ph.ref.assign(ph.N, Knot{});
    ph.par.assign(ph.N, Par{});
    ph.rc.assign(ph.N, RCost{});
    ph.ctg.assign(ph.N, CTG{});
    memset(ph.pc, 0, sizeof ph.pc);
    ph.Phi = 0;
    memset(ph.Phix, 0, sizeof ph.Phix);
    memset(ph.Phixx, 0, sizeof ph.Phixx);
    ph.h = 0;
    memset(ph.hx, 0, sizeof ph.hx);
    memset(ph.hxx, 0, sizeof ph.hxx);
    ph.V = ph.dV = ph.dVnext = 0;
    memset(ph.Gnext, 0, sizeof ph.Gnext);
    memset(ph.Hnext, 0, sizeof ph.Hnext);
    memset(ph.x0, 0, sizeof ph.x0);
    init_params(ph);
  }
  memset(P.x0, 0, sizeof P.x0);
  memcpy(P.x0, x0, sizeof(double) * P.ph[0].n);
  P.tconstr_violation = 0;  // uninitialised in the reference (B9); masked by iter_AL == 1
  generate_ref(P);
  // MHPCLocomotion::warmstart (:200-215)
  double xph[14];
  memcpy(xph, P.x0, sizeof xph);
  for (int p = 0; p < d->n_wb; ++p) {
    memcpy(P.ph[p].act[0].x, xph, sizeof xph);
    bounding_pd(P.ph[p]);
    if (p + 1 < d->n_wb) phase_transition(P, p, xph);
  }
  update_nominal(P);
}

void export_problem(const Problem& P, int b, const mhpc_problem_desc* d, double* X, double* U,
                    double* Y, double* K, double* DU, double* G, double* J, double* dV,
                    double* viol, double* Vp, double* dVp, int32_t* status, int32_t* trace,
                    int64_t* counters) {
  const int np = (int)P.ph.size();
  size_t lx = 0, lu = 0, lk = 0;
  for (int p = 0; p < np; ++p) {
    lx += (size_t)P.ph[p].N * P.ph[p].n;
    lu += (size_t)P.ph[p].N * 4;
    lk += (size_t)P.ph[p].N * 4 * P.ph[p].n;
  }
  size_t ox = b * lx, ou = b * lu, ok = b * lk;
  for (int p = 0; p < np; ++p) {
    const Phase& ph = P.ph[p];
    for (int k = 0; k < ph.N; ++k) {
      for (int i = 0; i < ph.n; ++i) {
        if (X) X[ox + i] = ph.nom[k].x[i];
        if (G) G[ox + i] = ph.ctg[k].G[i];
      }
      for (int i = 0; i < 4; ++i) {
        if (U) U[ou + i] = ph.nom[k].u[i];
        if (Y) Y[ou + i] = ph.nom[k].y[i];
        if (DU) DU[ou + i] = ph.ctg[k].du[i];
      }
      if (K) memcpy(K + ok, ph.ctg[k].K, sizeof(double) * 4 * ph.n);
      ox += ph.n;
      ou += 4;
      ok += 4 * ph.n;
    }
    if (Vp) Vp[b * np + p] = ph.V;
    if (dVp) dVp[b * np + p] = ph.dV;
  }
  (void)d;
  if (J) J[b] = P.actual_cost;
  if (dV) dV[b] = P.exp_cost_change;
  if (viol) viol[b] = P.tconstr_violation;
  if (status) status[b] = P.status;
  if (trace) {
    for (int i = 0; i < MHPC_TRACE_LEN; ++i) trace[b * MHPC_TRACE_LEN + i] = i < P.ntrace ? P.trace[i] : -1;
  }
  if (counters)
    for (int i = 0; i < 6; ++i) counters[b * 6 + i] = P.cnt[i];
}

}  // namespace

// One knot of SinglePhase::backward_sweep (SinglePhase.cpp:197-212) on caller-supplied
// blocks, exactly the body of phase_backward_sweep: compute_Qfunction, + reg on the Qxx / Quu
// diagonals, the PSD test of Quu - 1e-9 I, valuefunction_update.  Row-major A [n][n],
// B [n][4], C [4][n], D [4][4], lxx [n][n], lux [4][n], luu / lyy [4][4], Hn [n][n].
// Returns 1 (PSD, K / du / G / H / dV written) or 0 (not PSD, nothing written); tests only.
extern "C" int oracle_riccati_knot(int n, const double* A, const double* B, const double* C,
                                   const double* D, const double* lx, const double* lu,
                                   const double* ly, const double* lxx, const double* lux,
                                   const double* luu, const double* lyy, const double* Gn,
                                   const double* Hn, double reg, double* K, double* du,
                                   double* G, double* H, double* dV) {
  if (n < 1 || n > 14) return -1;
  Par p{};
  RCost rc{};
  CTG c{};
  memcpy(p.A, A, sizeof(double) * n * n);
  memcpy(p.B, B, sizeof(double) * n * 4);
  memcpy(p.C, C, sizeof(double) * 4 * n);
  memcpy(p.D, D, sizeof(double) * 16);
  memcpy(rc.lx, lx, sizeof(double) * n);
  memcpy(rc.lu, lu, sizeof(double) * 4);
  memcpy(rc.ly, ly, sizeof(double) * 4);
  memcpy(rc.lxx, lxx, sizeof(double) * n * n);
  memcpy(rc.lux, lux, sizeof(double) * 4 * n);
  memcpy(rc.luu, luu, sizeof(double) * 16);
  memcpy(rc.lyy, lyy, sizeof(double) * 16);
  compute_Qfunction(c, rc, p, Gn, Hn, n);
  for (int i = 0; i < n; ++i) c.Qxx[i * n + i] += 1.0 * reg;
  for (int i = 0; i < 4; ++i) c.Quu[i * 4 + i] += 1.0 * reg;
  double Qr[16];
  const double eps9 = pow(0.1, 9);
  for (int i = 0; i < 16; ++i) Qr[i] = c.Quu[i] - ((i % 5 == 0) ? 1.0 * eps9 : 0.0);
  if (!ldlt_is_positive(Qr, 4)) return 0;
  const double d = valuefunction_update(c, n);
  memcpy(K, c.K, sizeof(double) * 4 * n);
  memcpy(du, c.du, sizeof(double) * 4);
  memcpy(G, c.G, sizeof(double) * n);
  memcpy(H, c.H, sizeof(double) * n * n);
  *dV = d;
  return 1;
}

// Eigen::LDLT(A).isPositive() as the oracle restates it (row-major 4x4); tests only.
extern "C" int oracle_ldlt_is_positive(const double* A) { return ldlt_is_positive(A, 4) ? 1 : 0; }

// Counterpart of mhpc_set_cost_weights / mhpc_set_constraint_params for later oracle calls
// (NULL restores the reference's values); not thread-safe against a running solve.
extern "C" int oracle_set_params(const mhpc_cost_weights* w, const mhpc_constraint_params* c) {
  kWB = make_wb_weights();
  kFB = make_fb_weights();
  if (w) {
    for (int m = 0; m < 4; ++m) {
      for (int i = 0; i < 14; ++i) {
        kWB.Q[m][i] = w->wb_Q[m][i];
        kWB.Qf[m][i] = w->wb_Qf[m][i];
      }
      for (int i = 0; i < 4; ++i) {
        kWB.R[m][i] = w->wb_R[m][i];
        kWB.S[m][i] = w->wb_S[m][i];
        kFB.R[m][i] = w->fb_R[m][i];
      }
      for (int i = 0; i < 6; ++i) {
        kFB.Q[m][i] = w->fb_Q[m][i];
        kFB.Qf[m][i] = w->fb_Qf[m][i];
      }
    }
  }
  kCon = ConParams();
  if (c) {
    kCon.tq_lim = c->torque_limit;
    kCon.mu = c->friction_coeff;
    for (int m = 0; m < 4; ++m) {
      kCon.sigma[m] = c->sigma[m];
      kCon.delta[m] = c->delta[m];
      kCon.delta_min[m] = c->delta_min[m];
      kCon.eps_tq[m] = c->eps_torque[m];
      kCon.eps_grf[m] = c->eps_grf[m];
    }
  }
  return 0;
}

extern "C" int oracle_load_ref(const char* path) {
  if (g_ref.handle) return 0;
  g_ref.handle = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!g_ref.handle) return 1;
  bool ok = load_fn(g_ref.Dyn_FL, "Dyn_FL") && load_fn(g_ref.Dyn_BS, "Dyn_BS") &&
            load_fn(g_ref.Dyn_FS, "Dyn_FS") && load_fn(g_ref.Dyn_FL_par, "Dyn_FL_par") &&
            load_fn(g_ref.Dyn_BS_par, "Dyn_BS_par") && load_fn(g_ref.Dyn_FS_par, "Dyn_FS_par") &&
            load_fn(g_ref.Imp_F, "Imp_F") && load_fn(g_ref.Imp_B, "Imp_B") &&
            load_fn(g_ref.Imp_F_par, "Imp_F_par") && load_fn(g_ref.Imp_B_par, "Imp_B_par") &&
            load_fn(g_ref.FBDynamics, "FBDynamics") &&
            load_fn(g_ref.FBDynamics_par, "FBDynamics_par") &&
            load_fn(g_ref.WB_FL1, "WB_FL1_terminal_constr") &&
            load_fn(g_ref.WB_FL2, "WB_FL2_terminal_constr") && load_fn(g_ref.Jacob_F, "Jacob_F") &&
            load_fn(g_ref.Jacob_B, "Jacob_B");
  return ok ? 0 : 2;
}

extern "C" int oracle_solve(const mhpc_problem_desc* desc, const mhpc_hsddp_option* opt, int batch,
                            const double* x0, int nthreads, int do_solve, double* X, double* U,
                            double* Y, double* K, double* DU, double* G, double* J, double* dV,
                            double* viol, double* Vp, double* dVp, int32_t* status, int32_t* trace,
                            int64_t* counters) {
  if (!g_ref.handle) return 3;
  const int np = desc->n_wb + desc->n_fb;
  if (np < 1 || np > MHPC_MAX_PHASES) return 1;
  const int n0 = desc->n_wb > 0 ? 14 : 6;
  std::atomic<int> next(0);
  auto worker = [&]() {
    for (;;) {
      const int b = next.fetch_add(1);
      if (b >= batch) break;
      Problem P;
      build(P, desc, opt, x0 + (size_t)b * n0);
      if (do_solve) mp_solve(P);
      export_problem(P, b, desc, X, U, Y, K, DU, G, J, dV, viol, Vp, dVp, status, trace, counters);
    }
  };
  if (nthreads < 1) nthreads = 1;
  std::vector<std::thread> th;
  for (int t = 1; t < nthreads; ++t) th.emplace_back(worker);
  worker();
  for (auto& t : th) t.join();
  return 0;
}

// forward_sweep_dynamics_only at a list of step sizes from the state a solve leaves behind
// (nominal, gains, AL / ReB parameters): MultiPhaseDDP::forward_iteration's trial rollouts
// (MultiPhaseDDP.cpp:130-151) without the Armijo stop, for the C2 rollout workload.
// J / viol: [batch][n_eps].  do_solve = 0 evaluates right after initialization.
extern "C" int oracle_rollout_costs(const mhpc_problem_desc* desc, const mhpc_hsddp_option* opt,
                                    int batch, const double* x0, int nthreads, int do_solve,
                                    int n_eps, const double* eps, double* J, double* viol,
                                    double* rollout_seconds) {
  std::atomic<long long> ns(0);
  if (!g_ref.handle) return 3;
  const int np = desc->n_wb + desc->n_fb;
  if (np < 1 || np > MHPC_MAX_PHASES || n_eps < 1) return 1;
  const int n0 = desc->n_wb > 0 ? 14 : 6;
  std::atomic<int> next(0);
  auto worker = [&]() {
    for (;;) {
      const int b = next.fetch_add(1);
      if (b >= batch) break;
      Problem P;
      build(P, desc, opt, x0 + (size_t)b * n0);
      if (do_solve) mp_solve(P);
      const auto t0 = std::chrono::steady_clock::now();
      for (int e = 0; e < n_eps; ++e) {
        mp_forward_sweep(P, eps[e], true);
        J[(size_t)b * n_eps + e] = P.actual_cost;
        viol[(size_t)b * n_eps + e] = P.tconstr_violation;
      }
      ns += std::chrono::duration_cast<std::chrono::nanoseconds>(
                std::chrono::steady_clock::now() - t0).count();
    }
  };
  if (nthreads < 1) nthreads = 1;
  std::vector<std::thread> th;
  for (int t = 1; t < nthreads; ++t) th.emplace_back(worker);
  worker();
  for (auto& t : th) t.join();
  if (rollout_seconds) *rollout_seconds = ns.load() * 1e-9;  // summed over threads
  return 0;
}

// The cost gradients print_debugInfo writes to cost.txt (MHPCLocomotion.cpp:355-377) after
// a solve: rcost[k].lx of knots 0..N-2 and tcost.Phix of every phase, phase-concatenated:
// LX [batch][sum_p (N_p - 1) n_p], PHIX [batch][sum_p n_p].
extern "C" int oracle_cost_gradients(const mhpc_problem_desc* desc, const mhpc_hsddp_option* opt,
                                     int batch, const double* x0, int nthreads, double* LX,
                                     double* PHIX) {
  if (!g_ref.handle) return 3;
  const int np = desc->n_wb + desc->n_fb;
  if (np < 1 || np > MHPC_MAX_PHASES) return 1;
  const int n0 = desc->n_wb > 0 ? 14 : 6;
  std::atomic<int> next(0);
  auto worker = [&]() {
    for (;;) {
      const int b = next.fetch_add(1);
      if (b >= batch) break;
      Problem P;
      build(P, desc, opt, x0 + (size_t)b * n0);
      mp_solve(P);
      size_t llx = 0, lph = 0;
      for (const Phase& ph : P.ph) { llx += (size_t)(ph.N - 1) * ph.n; lph += ph.n; }
      double* lx = LX + (size_t)b * llx;
      double* phx = PHIX + (size_t)b * lph;
      for (const Phase& ph : P.ph) {
        for (int k = 0; k < ph.N - 1; ++k)
          for (int i = 0; i < ph.n; ++i) *lx++ = ph.rc[k].lx[i];
        for (int i = 0; i < ph.n; ++i) *phx++ = ph.Phix[i];
      }
    }
  };
  if (nthreads < 1) nthreads = 1;
  std::vector<std::thread> th;
  for (int t = 1; t < nthreads; ++t) th.emplace_back(worker);
  worker();
  for (auto& t : th) t.join();
  return 0;
}

// Receding-horizon loop (f2): initialization() + solve, then per tick set_initial_condition,
// MHPCLocomotion::update_problem (MHPCLocomotion.cpp:107-158) and solve again.  Phase
// buffers are emulated as the reference allocates them: one N_TIMESTEPS_MAX-knot buffer per
// WB and per SRB phase slot holding the nominal (ModelState) and cost-to-go (CTG); phases
// write through to their buffer, update_problem rotates which buffer each phase uses.
// x0s [ticks][batch][n0]; per tick: J, viol [ticks][batch], trace [ticks][batch][TRACE],
// N_out, modes_out [ticks][n_phases]; after the last tick the nominal X, U and K, G of every
// phase, phase-concatenated into X [batch][cap_x] etc. with cap = n_phases * 110 knots.
extern "C" int oracle_mpc(const mhpc_problem_desc* desc, const mhpc_hsddp_option* opt,
                          int n_modes, const int* gait_modes, const float* gait_timings,
                          int batch, int ticks, const double* x0s, int nthreads, double* J,
                          double* viol, int32_t* trace, int32_t* N_out, int32_t* modes_out,
                          double* X, double* U, double* K, double* G) {
  if (!g_ref.handle) return 3;
  const int np = desc->n_wb + desc->n_fb;
  if (np < 1 || np > MHPC_MAX_PHASES || ticks < 1 || n_modes < 1) return 1;
  const int n0 = desc->n_wb > 0 ? 14 : 6;
  constexpr int NBK = 110;  // N_TIMESTEPS_MAX
  std::atomic<int> next(0);
  std::atomic<int> err(0);
  auto next_mode = [&](int m) {
    for (int i = 0; i < n_modes; ++i)
      if (gait_modes[i] == m) return gait_modes[(i + 1) % n_modes];
    return -1;
  };
  auto worker = [&]() {
    for (;;) {
      const int b = next.fetch_add(1);
      if (b >= batch) break;
      mhpc_problem_desc dl = *desc;
      Problem P;
      // ms_act_*, ms_nom_*, CTG_* buffers (the act buffer matters: its last knot's u, y are
      // never written by a sweep and reach the nominal through update_nominal_trajectory)
      struct Buf { std::vector<Knot> act, nom; std::vector<CTG> ctg; };
      std::vector<Buf> bw(desc->n_wb), bf(desc->n_fb);
      for (auto& q : bw) { q.act.assign(NBK, Knot{}); q.nom.assign(NBK, Knot{}); q.ctg.assign(NBK, CTG{}); }
      for (auto& q : bf) { q.act.assign(NBK, Knot{}); q.nom.assign(NBK, Knot{}); q.ctg.assign(NBK, CTG{}); }
      std::vector<int> pw(desc->n_wb), pf(desc->n_fb);
      for (int i = 0; i < desc->n_wb; ++i) pw[i] = i;
      for (int i = 0; i < desc->n_fb; ++i) pf[i] = i;
      int cmode = dl.mode_seq[0];
      for (int t = 0; t < ticks; ++t) {
        const double* x0 = x0s + ((size_t)t * batch + b) * n0;
        if (t == 0) {
          build(P, &dl, opt, x0);
        } else {
          for (int p = 0; p < np; ++p) {  // phases wrote through to their buffers
            Buf& q = p < dl.n_wb ? bw[pw[p]] : bf[pf[p - dl.n_wb]];
            for (int k = 0; k < P.ph[p].N; ++k) {
              q.act[k] = P.ph[p].act[k];
              q.nom[k] = P.ph[p].nom[k];
              q.ctg[k] = P.ph[p].ctg[k];
            }
          }
          if (!pw.empty()) std::rotate(pw.begin(), pw.begin() + 1, pw.end());
          if (!pf.empty()) std::rotate(pf.begin(), pf.begin() + 1, pf.end());
          cmode = next_mode(cmode);
          if (cmode < 0) { err = 4; return; }
          dl.mode_seq[0] = cmode;
          for (int p = 1; p < np; ++p) dl.mode_seq[p] = next_mode(dl.mode_seq[p - 1]);
          for (int p = 0; p < np; ++p) {
            const double dt = p < dl.n_wb ? dl.dt_wb : dl.dt_fb;
            dl.N[p] = (int)round((double)gait_timings[dl.mode_seq[p] - 1] / dt);
            if (dl.N[p] < 2 || dl.N[p] > NBK) { err = 5; return; }
          }
          for (int p = 0; p < np; ++p) {  // set_phase_config + set_data + initialization
            Phase& ph = P.ph[p];
            Buf& q = p < dl.n_wb ? bw[pw[p]] : bf[pf[p - dl.n_wb]];
            ph.mode = dl.mode_seq[p];
            ph.N = dl.N[p];
            ph.act.assign(q.act.begin(), q.act.begin() + ph.N);
            ph.nom.assign(q.nom.begin(), q.nom.begin() + ph.N);
            ph.ref.assign(ph.N, Knot{});
            ph.par.assign(ph.N, Par{});
            ph.rc.assign(ph.N, RCost{});
            ph.ctg.assign(q.ctg.begin(), q.ctg.begin() + ph.N);
            init_params(ph);
          }
          memset(P.x0, 0, sizeof P.x0);
          memcpy(P.x0, x0, sizeof(double) * P.ph[0].n);
          generate_ref(P);
          P.status = MHPC_SOLVE_OK;
          P.ntrace = 0;
          for (int i = 0; i < 6; ++i) P.cnt[i] = 0;
        }
        for (int i = 0; i < MHPC_TRACE_LEN; ++i) P.trace[i] = -1;
        P.ntrace = 0;
        mp_solve(P);
        J[(size_t)t * batch + b] = P.actual_cost;
        viol[(size_t)t * batch + b] = P.tconstr_violation;
        memcpy(trace + ((size_t)t * batch + b) * MHPC_TRACE_LEN, P.trace,
               sizeof(int32_t) * MHPC_TRACE_LEN);
        if (b == 0)
          for (int p = 0; p < np; ++p) {
            N_out[t * np + p] = dl.N[p];
            modes_out[t * np + p] = dl.mode_seq[p];
          }
      }
      const size_t cap = (size_t)np * NBK;
      double* xo = X + (size_t)b * cap * 14;
      double* uo = U + (size_t)b * cap * 4;
      double* ko = K + (size_t)b * cap * 56;
      double* go = G + (size_t)b * cap * 14;
      for (const Phase& ph : P.ph)
        for (int k = 0; k < ph.N; ++k) {
          for (int i = 0; i < ph.n; ++i) *xo++ = ph.nom[k].x[i];
          for (int i = 0; i < 4; ++i) *uo++ = ph.nom[k].u[i];
          for (int i = 0; i < 4 * ph.n; ++i) *ko++ = ph.ctg[k].K[i];
          for (int i = 0; i < ph.n; ++i) *go++ = ph.ctg[k].G[i];
        }
    }
  };
  if (nthreads < 1) nthreads = 1;
  std::vector<std::thread> th;
  for (int t = 1; t < nthreads; ++t) th.emplace_back(worker);
  worker();
  for (auto& t : th) t.join();
  return err.load();
}
