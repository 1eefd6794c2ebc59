// k_bws: the backward Riccati sweep of the batched HSDDP solve, four problems per wavefront.
//
// Restates MultiPhaseDDP::backward_sweep + impact_aware_step (MultiPhaseDDP.cpp:100-127,
// 300-341), SinglePhase::backward_sweep (SinglePhase.cpp:183-216), compute_Qfunction and
// valuefunction_update (MHPC_CompoundTypes.h:117-144) and the regularisation retry loop of
// MultiPhaseDDP::solve (:196-241).
//
// Layout (round 4).  A problem owns one 16-lane row of a wave (DPP row); its value function
// and Q blocks live in registers, one matrix row per lane, and every product is a
// row-broadcast multiply-add, v_fmac_f64_dpp row_newbcast:L (mhpc_dpp.h): the multiplicand
// of lane L of the row reaches all 16 lanes inside the FMA, no LDS round trip.  The state
// (NX = 2 NQ: 14 whole-body, 6 SRB) has at most 16 rows, so one row of lanes holds a whole
// matrix.  Lane t of a row holds matrix row rho(t): the configuration rows q_i on the even
// lanes 2i, the velocity rows NQ + i on the odd lanes 2i + 1, control rows on the lanes after
// them (whole body: u0, u1 on lanes 14, 15, u2 / u3 as a second register set of lanes 14 / 15;
// SRB: u0..u3 on lanes 6..9).
//
// The dynamics Jacobian of a planar model with state (q, qdot) and explicit Euler has the
// shape
//     [A B] = [ I  dt*I  0 ]      (rows 0..NQ-1, exact)
//             [    W       ]      (rows NQ..NX-1: W = rows of I + dt*Ac | dt*Bc)
// so per knot, with H the value-function Hessian of knot k+1:
//   S = H [A B]          S[i][c] = a(c) H[i][b(c)] + sum_r H[i][NQ+r] W[r][c]
//                        (lane i: own H row, W[r][c] broadcast from the lane holding column c)
//   Q = [A B]' S + ...   Q[c][d] = a(c) S[b(c)][d] + sum_r W[r][c] S[NQ+r][d]
//                        (lane c: own W column, S[NQ+r][d] broadcast from lane 2r+1; the
//                        a-term S[b(c)][d] of a velocity row is the configuration row on the
//                        lane below: one quad_perm DPP move)
// with a(c), b(c) = 1, c / dt, c - NQ / 0 for configuration / velocity / control columns.
// C and D (stance rows of the contact forces) enter as rank-2 updates with broadcast rows.
// Every lane of a row runs the same instruction stream; lanes that hold no matrix row compute
// finite filler that no real row reads.
//
// The 4x4 control block is assembled on every lane (row broadcasts), tested for
// positive-definiteness (unpivoted LDL^T of Quu - 1e-9 I, tests/test_psd_verdict.py) and
// applied through its own LDL^T factor; Q is symmetric by construction in its control block
// and Qxx is symmetrised through one LDS transpose per knot, as the reference does
// (MHPC_CompoundTypes.h:133-134).
// The arithmetic is the reference's up to summation order (parity: tests/test_gpu_solve.py);
// every launch shape (problems per wave) runs the same per-row code, so all of them agree bit
// for bit (tests/test_gpu_variants.py).
#include <hip/hip_runtime.h>

#include <type_traits>
#include <utility>

#include "mhpc_device.h"
#include "mhpc_dpp.h"

namespace MHPC_NS {
int launch_problems(const SolveParams& sp);  // mhpc_kernels.hip
// MHPC_BWS_VARIANT_NS: a second instantiation of this file in one library (the fp32 library's
// float sweep, MHPC_BWS_F64=0) lives in a nested namespace -- its kernels and entry points
// (launch_bws, bws_split, bws_auto_variant) do not collide with the default build's.
#ifdef MHPC_BWS_VARIANT_NS
namespace MHPC_BWS_VARIANT_NS {
#endif

// Arithmetic type of the whole-body knots' 4x4 control block (inverse, gains, and the H / G /
// dV updates with them): the solve's type, or double in the fp32 build (MHPC_BWS_WIDE,
// default): the fp32 sweep's gains then carry the rounding of the fp32 Q blocks only, not of
// an fp32 inversion (tools/diag_fp32_stages.py).
#ifndef MHPC_BWS_WIDE
#define MHPC_BWS_WIDE 1
#endif
// Arithmetic type of the whole sweep (MHPC_BWS_F64, default): double in both builds.  The fp32
// build reads its float records and writes float gains, but sums, factors and carries the
// value function in double -- on MI355X an fp64 FMA issues at the fp32 rate (no packed math in
// this code), so the fp32 sweep was never faster than the fp64 one, and its rounding was the
// largest source of the fp32 solve's error (tools/diag_fp32_stages.py; round 6: the round-5
// codegen change that moved one ill-conditioned C5 problem's G error from 2.5e-2 to 6.2e-2 was
// rounding of the fp32 sweep, tools/fp32_bisect.py).  Built with -DMHPC_BWS_F64=0 the fp32
// sweep computes in float with the control block in double (MHPC_BWS_WIDE), as in round 5.
#ifndef MHPC_BWS_F64
#define MHPC_BWS_F64 1
#endif
#if defined(MHPC_FP32) && MHPC_BWS_F64
using breal = double;
#else
using breal = real;
#endif
#if defined(MHPC_FP32) && MHPC_BWS_WIDE
using wreal = double;
#else
using wreal = breal;
#endif

template <int I>
using ic = std::integral_constant<int, I>;
template <int A, int B, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (A < B) {
    f(ic<A>{});
    sfor<A + 1, B>(f);
  }
}

// Lane maps of one 16-lane row (see the file header).
template <int NQ>
struct Rows {
  static constexpr int NX = 2 * NQ, NC = NX + 4;
  // matrix row held by lane t (t >= NC: none; such lanes clamp their addresses)
  static constexpr __host__ __device__ int rho(int t) {
    return t < NX ? ((t & 1) ? NQ + (t >> 1) : (t >> 1)) : t;
  }
  // lane holding matrix row / column i (whole body: 16, 17 are the second set of 14, 15)
  static constexpr __host__ __device__ int lam(int i) {
    return i < NQ ? 2 * i : i < NX ? 2 * (i - NQ) + 1 : i < 16 ? i : 14 + (i - 16);
  }
};

// Value of lane K of this lane's 16-lane row.
template <int K>
__device__ __forceinline__ double rbc(double v) {
  return __builtin_amdgcn_update_dpp(v, v, 0x150 + K, 0xf, 0xf, true);
}
template <int K>
__device__ __forceinline__ float rbc(float v) {
  return __builtin_amdgcn_update_dpp(v, v, 0x150 + K, 0xf, 0xf, true);
}
// quad_perm [0,0,2,2]: an odd lane takes the value of the even lane below it (the
// configuration row matching a velocity row), an even lane keeps its own.
__device__ __forceinline__ int qperm_i(int v) {
  return __builtin_amdgcn_update_dpp(v, v, 0xA0, 0xf, 0xf, true);
}
__device__ __forceinline__ double qperm(double v) {
  return __hiloint2double(qperm_i(__double2hiint(v)), qperm_i(__double2loint(v)));
}
__device__ __forceinline__ float qperm(float v) { return __int_as_float(qperm_i(__float_as_int(v))); }
// Two-row layout: on rows 1 and 3 (row B of a problem) an even lane takes the odd lane above
// it (quad_perm [1,1,3,3], row_mask 0b1010); rows 0 and 2 keep their own value.
__device__ __forceinline__ int qshift_rowB_i(int v) {
  return __builtin_amdgcn_update_dpp(v, v, 0xF5, 0xA, 0xF, false);
}
__device__ __forceinline__ double qshift_rowB(double v) {
  return __hiloint2double(qshift_rowB_i(__double2hiint(v)), qshift_rowB_i(__double2loint(v)));
}
__device__ __forceinline__ float qshift_rowB(float v) {
  return __int_as_float(qshift_rowB_i(__float_as_int(v)));
}
// Row pair exchange (v_permlane16_swap): a = row A's value, b = row B's value, on both rows.
__device__ __forceinline__ void row_pair_swap_i(unsigned v, unsigned& a, unsigned& b) {
  const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  a = r[0];
  b = r[1];
}
__device__ __forceinline__ void row_pair_swap(double v, double& a, double& b) {
  unsigned ahi, bhi, alo, blo;
  row_pair_swap_i((unsigned)__double2hiint(v), ahi, bhi);
  row_pair_swap_i((unsigned)__double2loint(v), alo, blo);
  a = __hiloint2double((int)ahi, (int)alo);
  b = __hiloint2double((int)bhi, (int)blo);
}
__device__ __forceinline__ void row_pair_swap(float v, float& a, float& b) {
  unsigned ua, ub;
  row_pair_swap_i((unsigned)__float_as_int(v), ua, ub);
  a = __int_as_float((int)ua);
  b = __int_as_float((int)ub);
}

// 1 / a by the hardware estimate and two Newton steps (within an ulp of the division; the
// IEEE division sequence is twice the instructions and latency)
__device__ __forceinline__ double recip(double a) {
  double r = __builtin_amdgcn_rcp(a);
  double e = __builtin_fma(-a, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-a, r, 1.0);
  return __builtin_fma(r, e, r);
}
__device__ __forceinline__ float recip(float a) {
  float r = __builtin_amdgcn_rcpf(a);
  const float e = __builtin_fmaf(-a, r, 1.0f);
  return __builtin_fmaf(r, e, r);
}

// Eigen::LDLT(Quu - 1e-9 I).isPositive() (SinglePhase.cpp:202-209): an unpivoted LDL^T of
// the lower triangle.  By Sylvester's law of inertia its pivots have the signs of Eigen's
// pivoted factorisation's whenever no pivot is exactly zero, so the verdict is the same; a
// zero pivot leaves its column, as in Eigen (tests/test_psd_verdict.py).
__device__ __forceinline__ bool ldlt_nopiv_is_positive4(breal* A) {
  bool neg = false;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const breal akk = A[k * 5];
    neg = neg || akk < breal(0.0);
    // a zero pivot leaves its column (r = 0: the updates subtract exact zeros)
    const breal r = akk != breal(0.0) ? recip(akk) : breal(0.0);
#pragma unroll
    for (int i = k + 1; i < 4; ++i) {
      const breal l = A[i * 4 + k] * r;
#pragma unroll
      for (int j = k + 1; j <= i; ++j) A[i * 4 + j] -= l * A[j * 4 + k];
    }
  }
  return !neg;
}

// Quu^-1 applied by an LDL^T factorisation of the symmetric 4x4 control block (no explicit
// inverse: the reference forms (Quu^-1 + Quu^-T) / 2 and multiplies, MHPC_CompoundTypes.h
// :133-139; the factor solves the same systems -- up to rounding -- in about half the
// instructions).  Only used when Quu - 1e-9 I passed the PSD test, so the pivots are > 0.
template <class T>
struct Ldl4 {
  T l10, l20, l30, l21, l31, l32, r0, r1, r2, r3;  // unit lower factor, 1 / pivots
  __device__ __forceinline__ explicit Ldl4(const T (&q)[4][4]) {
    r0 = recip(q[0][0]);
    l10 = q[1][0] * r0;
    l20 = q[2][0] * r0;
    l30 = q[3][0] * r0;
    r1 = recip(q[1][1] - l10 * q[1][0]);
    const T u21 = q[2][1] - l20 * q[1][0], u31 = q[3][1] - l30 * q[1][0];
    l21 = u21 * r1;
    l31 = u31 * r1;
    r2 = recip((q[2][2] - l20 * q[2][0]) - l21 * u21);
    const T u32 = (q[3][2] - l30 * q[2][0]) - l31 * u21;
    l32 = u32 * r2;
    r3 = recip(((q[3][3] - l30 * q[3][0]) - l31 * u31) - l32 * u32);
  }
  // The same factorisation with the PSD test folded in (round 6).  ldlt_nopiv_is_positive4 on
  // Quu - eps I runs exactly these operations on exactly these entries (its elimination order
  // is this one's), so one instruction stream does both: every lane factors Quu for the solve
  // except the lane where psd_lane holds, which factors Quu - shift I with the test's zero-pivot
  // rule and returns its verdict in neg (pivot < 0).  That lane must hold no matrix row the knot
  // needs (its K, du, H are garbage, but finite).  One factorisation per knot instead of two.
  __device__ __forceinline__ Ldl4(const T (&q)[4][4], T shift, bool psd_lane, bool& neg) {
    auto piv = [&](T a) { return (a != T(0.0) || !psd_lane) ? recip(a) : T(0.0); };
    const T a00 = q[0][0] - shift;
    r0 = piv(a00);
    l10 = q[1][0] * r0;
    l20 = q[2][0] * r0;
    l30 = q[3][0] * r0;
    const T a11 = (q[1][1] - shift) - l10 * q[1][0];
    r1 = piv(a11);
    const T u21 = q[2][1] - l20 * q[1][0], u31 = q[3][1] - l30 * q[1][0];
    l21 = u21 * r1;
    l31 = u31 * r1;
    const T a22 = ((q[2][2] - shift) - l20 * q[2][0]) - l21 * u21;
    r2 = piv(a22);
    const T u32 = (q[3][2] - l30 * q[2][0]) - l31 * u21;
    l32 = u32 * r2;
    const T a33 = (((q[3][3] - shift) - l30 * q[3][0]) - l31 * u31) - l32 * u32;
    r3 = piv(a33);
    neg = a00 < T(0.0) || a11 < T(0.0) || a22 < T(0.0) || a33 < T(0.0);
  }
  // x = -Quu^-1 b
  __device__ __forceinline__ void neg_solve(const T (&b)[4], T (&x)[4]) const {
    const T z0 = b[0];
    const T z1 = b[1] - l10 * z0;
    const T z2 = (b[2] - l20 * z0) - l21 * z1;
    const T z3 = ((b[3] - l30 * z0) - l31 * z1) - l32 * z2;
    const T w0 = -(z0 * r0), w1 = -(z1 * r1), w2 = -(z2 * r2), w3 = -(z3 * r3);
    x[3] = w3;
    x[2] = w2 - l32 * x[3];
    x[1] = (w1 - l21 * x[2]) - l31 * x[3];
    x[0] = ((w0 - l10 * x[1]) - l20 * x[2]) - l30 * x[3];
  }
};

// The knot's control block: factor for the solve and the PSD verdict of
// Eigen::LDLT(Quu - 1e-9 I).isPositive() (SinglePhase.cpp:202-209), row-uniform.  Lane 15 of
// each 16-lane row runs the PSD test inside the shared factorisation (Ldl4 above): it is an
// SRB row's filler lane, or the whole-body sweep's second control lane, whose K and H rows are
// never stored or broadcast.  MHPC_BWS_PSD_SEPARATE=1: the test as its own factorisation (the
// round-5 form; same verdicts and factors bit for bit, tests/test_gpu_variants.py).
#ifndef MHPC_BWS_PSD_SEPARATE
#define MHPC_BWS_PSD_SEPARATE 1
#endif
template <class W>
__device__ __forceinline__ Ldl4<W> control_factor(const W (&q)[4][4], breal eps9, int t, bool& psd) {
  if constexpr (MHPC_BWS_PSD_SEPARATE || !std::is_same<W, breal>::value) {
    breal A[16];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) A[a * 4 + c] = breal(q[a][c]) - (a == c ? eps9 : breal(0.0));
    psd = ldlt_nopiv_is_positive4(A);
    return Ldl4<W>(q);
  } else {
    const bool pl = t == 15;
    bool neg;
    const Ldl4<W> F(q, pl ? W(eps9) : W(0.0), pl, neg);
    // lane 15's verdict to its row (row_newbcast:15)
    psd = __builtin_amdgcn_update_dpp(0, neg ? 1 : 0, 0x150 + 15, 0xf, 0xf, false) == 0;
    return F;
  }
}

// Ordering point of this wave's LDS accesses for the Qxx transpose: every row's writes (and
// the diagonal's atomic add) before the reads of the other rows' columns, and those reads
// before the next knot's writes.  One wave's LDS operations complete in issue order, so the
// hardware needs no wait here; the compiler must only keep the order.  Wavefront-scope fences
// generate no instruction (AMDGPU memory model) but are acquire / release points of the C++
// model, and the wave barrier keeps memory operations from moving across.
__device__ __forceinline__ void wave_lds_order() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Per-row LDS: the knot's Q rows for the Qxx transpose, and the value function at phase
// boundaries; entry (r, c) of the 16 x 16 block at M[at(r, c)].
//
// Default (round 5): row-major, pitch MP reals (16-byte aligned rows: the compiler writes a row
// with ds_write_b128 and reads a transposed column as ds_read2_b64 pairs).  Rows rho and
// rho + 8 share banks in the 8-lane groups of ds_write_b128, so 34 % of the WB sweep's LDS-array
// cycles are bank conflicts (profiles/r05_sq_counters_b1024.txt).
//
// MHPC_LDS_COLMAJOR=1 (round 6): column-major with pitch 18 and the RowLds of adjacent problems
// an odd number of reals apart; row writes (lane rho stores (rho, j); 16-lane groups over 32
// banks) touch 16 consecutive words, and a transposed read issued as one ds_read_b64 per value
// (32-lane groups over 64 banks: one row's 16 columns on 16 distinct even word slots, the
// other half of the group on odd slots) is conflict-free -- the reads go through lds_single,
// since the ds_read2_b64 pairs the compiler would merge them into conflict 2-way.  Measured
// (profiles/r06_lds_layout_ab.txt): conflict cycles 34 % -> 0.8 % of the LDS-array cycles of
// k_bws<2,2,2> and half the LDS-array cycles, all outputs bitwise equal -- but the WB half is
// 1.2 % slower at batch 1024 and the one-row sweep 3.7 % slower in C5 at 4096: seven (fourteen)
// single reads per knot instead of four (seven) paired ones cost more issue slots than the
// conflicts cost LDS cycles in this latency-bound loop.  So it is not the default.
#ifndef MHPC_LDS_COLMAJOR
#define MHPC_LDS_COLMAJOR 0
#endif
#if MHPC_LDS_COLMAJOR
constexpr int MP = 18;
__device__ __forceinline__ constexpr int at(int r, int c) { return c * MP + r; }
struct RowLds {
  breal M[16 * MP];
  breal Gs[16];
  breal hx[14], Hs[9], h;
  breal pad;  // odd size (329 reals)
};
static_assert(sizeof(RowLds) == 329 * sizeof(breal), "RowLds must stay an odd number of reals");
#else
constexpr int MP = sizeof(breal) == 8 ? 18 : 20;
__device__ __forceinline__ constexpr int at(int r, int c) { return r * MP + c; }
struct RowLds {
  alignas(16) breal M[16 * MP];
  breal Gs[16];
  breal hx[14], Hs[9], h;
};
#endif

typedef __attribute__((address_space(3))) const breal lds_creal;
// Read q[j] of the LDS block.  Column-major layout: as one single-word read -- the pointer
// passes through an empty asm first (no instruction), so the compiler cannot merge it with the
// neighbouring reads into a ds_read2 / b128; the caller threads the pointer into the next read,
// so no copy of the address register is needed.
__device__ __forceinline__ breal lds_single(lds_creal*& q, int j) {
  if (MHPC_LDS_COLMAJOR) asm volatile("" : "+v"(q));
  return q[j];
}
struct BwsLds {
  RowLds r[4];
};

// What one lane knows about its row's problem.
struct RowCtx {
  int b;       // problem (clamped into the batch for a spare row)
  int t;       // lane within the row
  int rp;      // row of the problem this lane's row is (0, or 1 in the two-row layout)
  int lt, nl;  // lane within the problem's rows, lanes per problem (16 or 32)
  bool act;    // the row holds an active problem in this launch
  bool live;   // the row takes part in the current sweep attempt
  bool failed; // ... and its attempt has failed (PSD test) -- sticky for the attempt
  int nom;     // nominal trajectory slot
  breal reg;    // regularisation of the attempt
  acc dV;      // expected cost change (row-uniform)
  int64_t kn, kn_wb, px_reads;
};

__device__ __forceinline__ bool go(const RowCtx& r) { return r.live && !r.failed; }

// Outputs of a knot awaiting their store.
struct PendingKnot {
  bool ok;
  int k;
  breal K[4], du[4], G;
};
__device__ __forceinline__ bool any_go(const RowCtx& r) {
  return __builtin_amdgcn_ballot_w64(go(r)) != 0;
}

// ---------------------------------------------------------------------------------------
// Whole-body phase (NQ = 7): knots N-2..0 from the value function in rl.M / rl.Gs (H, G of
// knot N-1), result (knot 0) written back there.
//
// Per knot the partials record (mhpc_solver.h: 18 columns x (7 qddot rows + 2 force rows),
// then lu, luu, ly, lyy) is read straight into the lanes that own its columns; the next
// knot's record is loaded while the current one computes.
// Optional cycle accounting of the sweep (build with -DMHPC_BWS_TIMING, read with
// mhpc_dbg_bws_cycles, tools/bws_timing.py; lane 0 of every wave): 0 / 1 WB knot loops and
// knots, 2 / 3 SRB knot loops and knots, 4 terminal values, 5 impact steps, 6 kernel, 7 waves;
// 8..12 the SRB knot's segments (operands and output stores issued; S and Q; the Qxx
// transpose through LDS; the 4x4 control block: PSD test, factor, du, K, G; the value update
// and the loop test).  Each probe is an s_memtime + wait, so the segments add up to more than
// an uninstrumented knot (~250 cycles per probe) and LDS waits land in the segment that issued the
// operations.
#ifdef MHPC_BWS_TIMING
__device__ unsigned long long g_bws_cyc[16];
#define BWS_T(v) const unsigned long long v = threadIdx.x == 0 ? clock64() : 0ull
#define BWS_ADD(i, v) do { if (threadIdx.x == 0) atomicAdd(&g_bws_cyc[i], (unsigned long long)(v)); } while (0)
// (segments accumulate per wave in registers, added to the counters once per phase: an atomic
// per knot and segment from every wave serialised the timed loop behind the L2 atomics)
#define BWS_SEG(i, a, b) BWS_T(b); segacc[(i) - 8] += (b) - (a)
#else
#define BWS_T(v) do { } while (0)
#define BWS_ADD(i, v) do { } while (0)
#define BWS_SEG(i, a, b) do { } while (0)
#endif
// knot iterations a sweep function ran: only the timing build keeps the count
#ifdef MHPC_BWS_TIMING
#define BWS_ITERS(n) (n)
#else
#define BWS_ITERS(n) 0
#endif

template <bool STANCE>
__device__ int sweep_wb(const SolveParams& sp, const DevBufs& d, const Layout& L, const ProbState* st, RowLds& rl,
                         RowCtx& rc, int p) {
  using R = Rows<7>;
  using wk = wreal;
  const int t = rc.t, b = rc.b;
  const int N = L.N[p], ko = L.ko[p], mode = L.mode[p];
  const breal dt = L.dt[p];
  const int rho = R::rho(t);
  const bool xl = t < 14;
  const breal coef = xl ? ((t & 1) ? dt : breal(1.0)) : breal(0.0);
  // identity part of W: W[r][c] = dt * rec + (c == 7 + r)
  breal base[7];
#pragma unroll
  for (int r = 0; r < 7; ++r) base[r] = rho == 7 + r ? breal(1.0) : breal(0.0);
  // running-cost weight and fixed reference of state rho (CostBase.cpp:28-31)
  const int xi = xl ? rho : 0;
  const breal w2 = 2 * dt * sp.cw.wQ[mode - 1][xi];
  const breal rxc = xi == 1 ? sp.height : xi == 2 ? breal(0.0)
                   : (xi >= 3 && xi < 7) ? cQjointBias[xi - 3] : xi == 7 ? sp.vel : breal(0.0);
  // lxx + reg on the diagonal of Qxx (Ixx * regularisation): added twice to the transposed
  // copy in LDS, so that (Qxx + Qxx') / 2 carries it once
  const breal dg2 = xl ? 2 * (w2 + rc.reg) : breal(0.0);
  const real* pos = d.refpos + (size_t)b * sp.NK + ko;
  // prefetch registers (record of one knot): the lane's own column of [Ac Bc; C D], the
  // second control column set (lanes 14, 15), one cost derivative per lane (broadcast below)
  constexpr int NR = STANCE ? 9 : 7;  // rows of a record column read
  constexpr int NCS = STANCE ? 14 : 8;  // cost derivatives (lu, luu [, ly, lyy])
  // (in the record type: a float record converted at load time would make the compiler wait
  // for the load there, a knot early; converted at the use instead -- the same values)
  real pr1[NR], pr2[NR], pcv, pxn, ppos;
  const int c1 = rho;            // record column of W1 (0..15)
  const int c2 = 16 + (t & 1);   // second set: control columns 2, 3 (lanes 14, 15)
  const int cq = t < NCS ? t : 0;
  // (the nominal state first: the wait for the last load of a knot then never covers the
  // stores of the previous knot, which share gfx950's in-order VM counter)
  // the phase's operand bases (knot 0): a knot adds k times its record stride
  const real* tk0 = traj_ptr(sp, d, b, rc.nom, ko) + xi;
  const real* jc0 = d.par + par_jac(sp.NK, b, ko) + cq;
  const real* r10 = d.par + par_col(sp.NK, b, c1, ko);
  const real* r20 = d.par + par_col(sp.NK, b, c2, ko);
  auto load = [&](int k) {
    pxn = tk0[k * KS];
    ppos = pos[k];
    pcv = jc0[k * 14];
    const real* r1 = r10 + k * 9;
    const real* r2 = r20 + k * 9;
#pragma unroll
    for (int r = 0; r < NR; ++r) pr1[r] = r1[r];
#pragma unroll
    for (int r = 0; r < NR; ++r) pr2[r] = r2[r];
  };
  breal H[14], Gv;
  {
    const int hr = xl ? rho : 0;
#pragma unroll
    for (int j = 0; j < 14; ++j) H[j] = rl.M[at(hr, j)];
    Gv = rl.Gs[hr];
  }
  const int cr = rho;  // column of M read in the transpose (Qxu columns for lanes 14, 15)
  // The outputs (K, du, G) of a knot are stored one knot later, right before the next
  // prefetch: every global operation of a knot is then issued together after the wait for the
  // previous prefetch, and the next such wait (a knot later) finds the stores retired --
  // gfx950 counts loads and stores on one in-order VM counter.
  PendingKnot pend;
  pend.ok = false;
  const size_t rec0 = (size_t)b * sp.NK + ko;
  real* const K0 = d.K + rec0 * 56 + rho;
  real* const G0 = d.G + rec0 * 14 + rho;
  real* const du0 = d.du + rec0 * 4;
  auto store_pending = [&]() {
    if (pend.ok) {
      if (xl) {
#pragma unroll
        for (int a = 0; a < 4; ++a) K0[pend.k * 56 + a * 14] = pend.K[a];
        G0[pend.k * 14] = pend.G;
      } else if (t == 14) {
#pragma unroll
        for (int a = 0; a < 4; ++a) du0[pend.k * 4 + a] = pend.du[a];
      }
    }
    pend.ok = false;
  };
  if (N >= 2) load(N - 2);
  int it = 0;  // knot iterations the wave ran (the cycle accounting's knot count)
  for (int k = N - 2; k >= 0; --k) {
    ++it;
    // ---- the knot's derivatives (prefetched) ----
    breal W1[7], W2[7], G2o[2], G22[2];
#pragma unroll
    for (int r = 0; r < 7; ++r) W1[r] = __builtin_fma(breal(pr1[r]), dt, base[r]);
#pragma unroll
    for (int r = 0; r < 7; ++r) W2[r] = __builtin_fma(breal(pr2[r]), dt, breal(0.0));
    // C, D rows: copied out of the prefetch registers (a fresh value each, so the prefetch
    // buffer is dead before it is reloaded; a buffer live across its own reload costs a copy
    // at the back edge that waits for every outstanding memory operation, stores included)
    G2o[0] = G2o[1] = G22[0] = G22[1] = breal(0.0);
    if (STANCE) {
      asm volatile("" : "=v"(G2o[0]) : "0"(breal(pr1[NR - 2])));
      asm volatile("" : "=v"(G2o[1]) : "0"(breal(pr1[NR - 1])));
      asm volatile("" : "=v"(G22[0]) : "0"(breal(pr2[NR - 2])));
      asm volatile("" : "=v"(G22[1]) : "0"(breal(pr2[NR - 1])));
    }
    // cost derivatives: lane q of the row holds entry q of (lu, luu, ly, lyy)
    breal luu[4], ly[2] = {0, 0}, lyy[4] = {0, 0, 0, 0};
    const breal pcvd = pcv;
    const breal lu0 = rbc<0>(pcvd), lu1 = rbc<1>(pcvd), lu2 = rbc<2>(pcvd), lu3 = rbc<3>(pcvd);
    luu[0] = rbc<4>(pcvd); luu[1] = rbc<5>(pcvd); luu[2] = rbc<6>(pcvd); luu[3] = rbc<7>(pcvd);
    if (STANCE) {
      ly[0] = rbc<8>(pcvd); ly[1] = rbc<9>(pcvd);
      lyy[0] = rbc<10>(pcvd); lyy[1] = rbc<11>(pcvd); lyy[2] = rbc<12>(pcvd); lyy[3] = rbc<13>(pcvd);
    }
    const breal rxi = rho == 0 ? breal(ppos) : rxc;
    const breal lx = w2 * (breal(pxn) - rxi);
    const breal lu01 = (t & 1) ? lu1 : lu0;
    const breal l1 = xl ? lx : lu01;
    const breal l2 = (t & 1) ? lu3 : lu2;
    const bool gate = go(rc);
    rc.kn += gate ? 1 : 0;
    rc.kn_wb += gate ? 1 : 0;
    // everything derived from the prefetch registers before they are reloaded: the loads
    // (memory operations) stay behind these volatile statements, so the buffers of knot k
    // and k - 1 share registers (no copy of a loop-carried buffer at the back edge)
    asm volatile("" ::"v"(W1[0]), "v"(W1[1]), "v"(W1[2]), "v"(W1[3]), "v"(W1[4]), "v"(W1[5]),
                 "v"(W1[6]), "v"(W2[0]), "v"(W2[1]), "v"(W2[2]), "v"(W2[3]), "v"(W2[4]),
                 "v"(W2[5]), "v"(W2[6]), "v"(l1), "v"(l2));
    asm volatile("" ::"v"(G2o[0]), "v"(G2o[1]), "v"(G22[0]), "v"(G22[1]), "v"(luu[0]),
                 "v"(luu[1]), "v"(luu[2]), "v"(luu[3]), "v"(ly[0]), "v"(ly[1]), "v"(lyy[0]),
                 "v"(lyy[1]), "v"(lyy[2]), "v"(lyy[3]));
    store_pending();
    if (k > 0) load(k - 1);

    // ---- S = H [A B] (lane: row rho of S) and Q = [A B]' S + ... (lane: row rho of Q),
    // column block by column block (a Q column needs only its S column) ----
    breal S[18], Q[18], Q2[2], Qv1, Qv2;
#pragma unroll
    for (int c = 0; c < 7; ++c) S[c] = H[c];
#pragma unroll
    for (int c = 7; c < 14; ++c) S[c] = dt * H[c - 7];
#pragma unroll
    for (int c = 14; c < 18; ++c) S[c] = breal(0.0);
    breal cc[2] = {0, 0}, cc2[2] = {0, 0};
    if (STANCE) {
      // C' lyy C etc.: cc[z] = sum_y G2[y][rho] lyy[y][z], then Q[.][d] += sum_z cc[z] G2[z][d]
#pragma unroll
      for (int z = 0; z < 2; ++z) {
        cc[z] = G2o[0] * lyy[z] + G2o[1] * lyy[2 + z];
        cc2[z] = G22[0] * lyy[z] + G22[1] * lyy[2 + z];
      }
    }
    // column blocks 0..5, 6..11, 12..17: S block, then the Q block it feeds
    wb_s_a(S[0], S[1], S[2], S[3], S[4], S[5], W1, W2, H + 7);
#pragma unroll
    for (int c = 0; c < 6; ++c) Q[c] = coef * qperm(S[c]);
    sb_odd7_6(Q[0], Q[1], Q[2], Q[3], Q[4], Q[5], S + 0, W1);
    if (STANCE) wb_st_a(Q[0], Q[1], Q[2], Q[3], Q[4], Q[5], G2o, cc);
    wb_s_b(S[6], S[7], S[8], S[9], S[10], S[11], W1, W2, H + 7);
#pragma unroll
    for (int c = 6; c < 12; ++c) Q[c] = coef * qperm(S[c]);
    sb_odd7_6(Q[6], Q[7], Q[8], Q[9], Q[10], Q[11], S + 6, W1);
    if (STANCE) wb_st_b(Q[6], Q[7], Q[8], Q[9], Q[10], Q[11], G2o, cc);
    wb_s_c(S[12], S[13], S[14], S[15], S[16], S[17], W1, W2, H + 7);
#pragma unroll
    for (int c = 12; c < 18; ++c) Q[c] = coef * qperm(S[c]);
    Qv1 = __builtin_fma(coef, qperm(Gv), l1);
    Q2[0] = breal(0.0);
    Q2[1] = breal(0.0);
    Qv2 = l2;
    {
      const breal sc[7] = {S[12], S[13], S[14], S[15], S[16], S[17], Gv};
      sb_odd7_7(Q[12], Q[13], Q[14], Q[15], Q[16], Q[17], Qv1, sc, W1);
      // control rows 2, 3 (second set of lanes 14, 15): only their control columns
      const breal s2[3] = {S[16], S[17], Gv};
      sb_odd7_3(Q2[0], Q2[1], Qv2, s2, W2);
    }
    if (STANCE) {
      wb_st_c(Q[12], Q[13], Q[14], Q[15], Q[16], Q[17], Q2[0], Q2[1], G2o, G22, cc, cc2);
      Qv1 = (Qv1 + G2o[0] * ly[0]) + G2o[1] * ly[1];
      Qv2 = (Qv2 + G22[0] * ly[0]) + G22[1] * ly[1];
    }

    // ---- Qxx transpose through LDS (symmetrisation, MHPC_CompoundTypes.h:134) ----
#pragma unroll
    for (int j = 0; j < 16; ++j) rl.M[at(rho, j)] = Q[j];
    // + 2 (lxx + reg) on the diagonal of the transposed copy: an LDS atomic add, in order with
    // this wave's other LDS operations, no round trip
    atomicAdd(&rl.M[at(rho, rho)], dg2);
    wave_lds_order();
    breal T[14];
    {
      lds_creal* tq = (lds_creal*)&rl.M[at(0, cr)];
#pragma unroll
      for (int j = 0; j < 14; ++j) T[j] = lds_single(tq, at(j, 0));
    }
    wave_lds_order();

    // ---- the control block on every lane ----
    wk q[4][4], Qu[4];
    q[0][0] = rbc<14>(Q[14]); q[0][1] = rbc<14>(Q[15]); q[0][2] = rbc<14>(Q[16]); q[0][3] = rbc<14>(Q[17]);
    q[1][1] = rbc<15>(Q[15]); q[1][2] = rbc<15>(Q[16]); q[1][3] = rbc<15>(Q[17]);
    q[2][2] = rbc<14>(Q2[0]); q[2][3] = rbc<14>(Q2[1]); q[3][3] = rbc<15>(Q2[1]);
    Qu[0] = rbc<14>(Qv1); Qu[1] = rbc<15>(Qv1); Qu[2] = rbc<14>(Qv2); Qu[3] = rbc<15>(Qv2);
    // luu + reg on the diagonal (Iuu * regularisation)
#pragma unroll
    for (int a = 0; a < 4; ++a) q[a][a] = q[a][a] + wk(luu[a] + rc.reg);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < a; ++c) q[a][c] = q[c][a];
    bool psd;
    const Ldl4<wk> F = control_factor<wk>(q, sp.eps9, t, psd);
    // du = -Quu^-1 Qu, dV += -Qu' Quu^-1 Qu (no 1/2, MHPC_CompoundTypes.h:137-142)
    wk du[4], dv = wk(0.0);
    F.neg_solve(Qu, du);
#pragma unroll
    for (int a = 0; a < 4; ++a) dv += Qu[a] * du[a];
    // K = -Quu^-1 Qux: column rho on lane rho (Qux[m][rho] = Q[rho][14 + m], own)
    wk Qxu[4], K[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) Qxu[m] = wk(Q[14 + m]);
    F.neg_solve(Qxu, K);
    // G = Qx - Qux' Quu^-1 Qu
    wk Gn = wk(Qv1);
#pragma unroll
    for (int a = 0; a < 4; ++a) Gn += K[a] * Qu[a];
    // H = sym(Qxx) - Qux' Quu^-1 Qux: H[rho][j] = Qs[j] + sum_a K[a] Qux[a][j]
    wk Hn[14];
#pragma unroll
    for (int j = 0; j < 14; ++j) Hn[j] = wk((Q[j] + T[j]) / 2);
    wb_h_a(Hn[0], Hn[1], Hn[2], Hn[3], Hn[4], Hn[5], Hn[6], Qxu, K);
    wb_h_b(Hn[7], Hn[8], Hn[9], Hn[10], Hn[11], Hn[12], Hn[13], Qxu, K);
#pragma unroll
    for (int j = 0; j < 14; ++j) H[j] = breal(Hn[j]);
    Gv = breal(Gn);
    // ---- outputs of knot k (only while the row's attempt is alive) ----
    const bool ok = gate && psd;
    // outputs of knot k, stored at the top of the next knot (see store_pending)
    pend.ok = ok;
    pend.k = k;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      pend.K[a] = breal(K[a]);
      pend.du[a] = breal(du[a]);
    }
    pend.G = breal(Gn);
    if (ok) rc.dV += acc(dv);
    rc.failed = rc.failed || (gate && !psd);
    if (!any_go(rc)) break;
  }
  store_pending();
  // value function of knot 0 back to LDS
  __syncthreads();
  if (xl) {
#pragma unroll
    for (int j = 0; j < 14; ++j) rl.M[at(rho, j)] = H[j];
    rl.Gs[rho] = Gv;
  }
  __syncthreads();
  return BWS_ITERS(it);
}

// ---------------------------------------------------------------------------------------
// Whole-body phase, two rows per problem (sweep_wb2, the launch shape for batches that leave
// SIMDs idle).  Both rows hold the value function (row rho(t) on lane t) and the control
// columns 14..17; row A computes the configuration columns 0..6 of S and Q, row B the
// velocity columns 7..13 in the same register slots.  Row B's broadcast copy of [A B] puts
// column 7 + s on lane 2 s, so both rows run the same instruction stream with the same DPP
// lane immediates (the S/Q blocks shrink from 18 + 1 to 11 + 1 columns per row).  The
// transpose writes each row's half of Qxx to the shared LDS block; each row updates its seven
// columns of H, and one v_permlane16_swap per word gives both rows the full rows of H.  Every
// entry is computed with the one-row sweep's operations in the same order, so the two
// layouts agree bit for bit (tests/test_gpu_variants.py).
template <bool STANCE>
__device__ int sweep_wb2(const SolveParams& sp, const DevBufs& d, const Layout& L, const ProbState* st, RowLds& rl,
                          RowCtx& rc, int p) {
  using R = Rows<7>;
  using wk = wreal;
  const int t = rc.t, b = rc.b, rp = rc.rp;
  const int N = L.N[p], ko = L.ko[p], mode = L.mode[p];
  const breal dt = L.dt[p];
  const int rho = R::rho(t);
  const bool xl = t < 14;
  const breal coef = xl ? ((t & 1) ? dt : breal(1.0)) : breal(0.0);
  const breal coefS = rp ? dt : breal(1.0);  // S init: column s (row A) / 7 + s (row B)
  // broadcast column of the lane: its own (row A, odd lanes, lanes 14 / 15) or, on row B's
  // even lanes 2 s, the velocity column 7 + s
  const int cb = (rp && xl && !(t & 1)) ? 7 + (t >> 1) : rho;
  breal base[7], baseb[7];
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    base[r] = rho == 7 + r ? breal(1.0) : breal(0.0);
    baseb[r] = cb == 7 + r ? breal(1.0) : breal(0.0);
  }
  const int xi = xl ? rho : 0;
  const breal w2 = 2 * dt * sp.cw.wQ[mode - 1][xi];
  const breal rxc = xi == 1 ? sp.height : xi == 2 ? breal(0.0)
                   : (xi >= 3 && xi < 7) ? cQjointBias[xi - 3] : xi == 7 ? sp.vel : breal(0.0);
  // lxx + reg on the diagonal, added by the row that owns the diagonal's column
  const bool own_diag = xl && ((rho < 7) == (rp == 0));
  const breal dg2 = own_diag ? 2 * (w2 + rc.reg) : breal(0.0);
  const real* pos = d.refpos + (size_t)b * sp.NK + ko;
  constexpr int NR = STANCE ? 9 : 7;
  constexpr int NCS = STANCE ? 14 : 8;
  real pr1[NR], prb[NR], pr2[NR], pcv, pxn, ppos;  // record type, see sweep_wb
  const int c2 = 16 + (t & 1);
  const int cq = t < NCS ? t : 0;
  // the phase's operand / output bases (knot 0): a knot adds k times its record stride
  const real* tk0 = traj_ptr(sp, d, b, rc.nom, ko) + xi;
  const real* jc0 = d.par + par_jac(sp.NK, b, ko) + cq;
  const real* r10 = d.par + par_col(sp.NK, b, rho, ko);
  const real* rb0 = d.par + par_col(sp.NK, b, cb, ko);
  const real* r20 = d.par + par_col(sp.NK, b, c2, ko);
  auto load = [&](int k) {
    pxn = tk0[k * KS];
    ppos = pos[k];
    pcv = jc0[k * 14];
    const real* r1 = r10 + k * 9;
    const real* rb = rb0 + k * 9;
    const real* r2 = r20 + k * 9;
#pragma unroll
    for (int r = 0; r < NR; ++r) pr1[r] = r1[r];
#pragma unroll
    for (int r = 0; r < NR; ++r) prb[r] = rb[r];
#pragma unroll
    for (int r = 0; r < NR; ++r) pr2[r] = r2[r];
  };
  breal H[14], Gv;
  {
    const int hr = xl ? rho : 0;
#pragma unroll
    for (int j = 0; j < 14; ++j) H[j] = rl.M[at(hr, j)];
    Gv = rl.Gs[hr];
  }
  // column read in the transpose; lanes 14, 15 (no row of Qxx) read column 0 with lane 0 (a
  // broadcast): columns 14, 15 are never written in this layout, and a filler lane's H row
  // still enters 0 * x products, so it must stay finite
  // row-major layout: matrix column c at LDS column mcol(c) (row B's half 16-byte aligned)
  auto mcol = [](int c) { return MHPC_LDS_COLMAJOR ? c : (c < 7 ? c : c + 1); };
  const int cr = xl ? mcol(rho) : 0;
  const int wo = rp ? mcol(7) : 0;      // LDS column of the row's first Q slot
  const int jr = rp ? 7 : 0;            // first matrix row of the row's H columns
  PendingKnot pend;
  pend.ok = false;
  const size_t rec0 = (size_t)b * sp.NK + ko;
  real* const K0 = d.K + rec0 * 56 + rho;
  real* const G0 = d.G + rec0 * 14 + rho;
  real* const du0 = d.du + rec0 * 4;
  auto store_pending = [&]() {
    if (pend.ok) {
      if (xl) {
#pragma unroll
        for (int a = 0; a < 4; ++a) K0[pend.k * 56 + a * 14] = pend.K[a];
        G0[pend.k * 14] = pend.G;
      } else if (t == 14) {
#pragma unroll
        for (int a = 0; a < 4; ++a) du0[pend.k * 4 + a] = pend.du[a];
      }
    }
    pend.ok = false;
  };
  if (N >= 2) load(N - 2);
  int it = 0;  // knot iterations the wave ran (the cycle accounting's knot count)
  for (int k = N - 2; k >= 0; --k) {
    ++it;
    breal Wo[7], Wb[7], W2[7], G2o[2], G2b[2], G22[2];
#pragma unroll
    for (int r = 0; r < 7; ++r) {
      Wo[r] = __builtin_fma(breal(pr1[r]), dt, base[r]);
      Wb[r] = __builtin_fma(breal(prb[r]), dt, baseb[r]);
      W2[r] = __builtin_fma(breal(pr2[r]), dt, breal(0.0));
    }
    G2o[0] = G2o[1] = G2b[0] = G2b[1] = G22[0] = G22[1] = breal(0.0);
    if (STANCE) {  // fresh values (see sweep_wb)
      asm volatile("" : "=v"(G2o[0]) : "0"(breal(pr1[NR - 2])));
      asm volatile("" : "=v"(G2o[1]) : "0"(breal(pr1[NR - 1])));
      asm volatile("" : "=v"(G2b[0]) : "0"(breal(prb[NR - 2])));
      asm volatile("" : "=v"(G2b[1]) : "0"(breal(prb[NR - 1])));
      asm volatile("" : "=v"(G22[0]) : "0"(breal(pr2[NR - 2])));
      asm volatile("" : "=v"(G22[1]) : "0"(breal(pr2[NR - 1])));
    }
    breal luu[4], ly[2] = {0, 0}, lyy[4] = {0, 0, 0, 0};
    const breal pcvd = pcv;
    const breal lu0 = rbc<0>(pcvd), lu1 = rbc<1>(pcvd), lu2 = rbc<2>(pcvd), lu3 = rbc<3>(pcvd);
    luu[0] = rbc<4>(pcvd); luu[1] = rbc<5>(pcvd); luu[2] = rbc<6>(pcvd); luu[3] = rbc<7>(pcvd);
    if (STANCE) {
      ly[0] = rbc<8>(pcvd); ly[1] = rbc<9>(pcvd);
      lyy[0] = rbc<10>(pcvd); lyy[1] = rbc<11>(pcvd); lyy[2] = rbc<12>(pcvd); lyy[3] = rbc<13>(pcvd);
    }
    const breal rxi = rho == 0 ? breal(ppos) : rxc;
    const breal lx = w2 * (breal(pxn) - rxi);
    const breal lu01 = (t & 1) ? lu1 : lu0;
    const breal l1 = xl ? lx : lu01;
    const breal l2 = (t & 1) ? lu3 : lu2;
    const bool gate = go(rc);
    rc.kn += gate ? 1 : 0;
    rc.kn_wb += gate ? 1 : 0;
    asm volatile("" ::"v"(Wo[0]), "v"(Wo[1]), "v"(Wo[2]), "v"(Wo[3]), "v"(Wo[4]), "v"(Wo[5]),
                 "v"(Wo[6]), "v"(Wb[0]), "v"(Wb[1]), "v"(Wb[2]), "v"(Wb[3]), "v"(Wb[4]),
                 "v"(Wb[5]), "v"(Wb[6]), "v"(l1), "v"(l2));
    asm volatile("" ::"v"(W2[0]), "v"(W2[1]), "v"(W2[2]), "v"(W2[3]), "v"(W2[4]), "v"(W2[5]),
                 "v"(W2[6]), "v"(G2o[0]), "v"(G2o[1]), "v"(G2b[0]), "v"(G2b[1]), "v"(G22[0]),
                 "v"(G22[1]));
    asm volatile("" ::"v"(luu[0]), "v"(luu[1]), "v"(luu[2]), "v"(luu[3]), "v"(ly[0]), "v"(ly[1]),
                 "v"(lyy[0]), "v"(lyy[1]), "v"(lyy[2]), "v"(lyy[3]));
    store_pending();
    if (k > 0) load(k - 1);

    // ---- S and Q, slots 0..6 (the row's half of columns 0..13) and 7..10 (columns 14..17)
    breal S[11], Q[11], Q2[2], Qv1, Qv2;
#pragma unroll
    for (int s = 0; s < 7; ++s) S[s] = coefS * H[s];
#pragma unroll
    for (int s = 7; s < 11; ++s) S[s] = breal(0.0);
    breal cc[2] = {0, 0}, cc2[2] = {0, 0};
    if (STANCE) {
#pragma unroll
      for (int z = 0; z < 2; ++z) {
        cc[z] = G2o[0] * lyy[z] + G2o[1] * lyy[2 + z];
        cc2[z] = G22[0] * lyy[z] + G22[1] * lyy[2 + z];
      }
    }
    wb_s_a(S[0], S[1], S[2], S[3], S[4], S[5], Wb, W2, H + 7);
#pragma unroll
    for (int s = 0; s < 6; ++s) Q[s] = coef * qperm(S[s]);
    sb_odd7_6(Q[0], Q[1], Q[2], Q[3], Q[4], Q[5], S + 0, Wo);
    if (STANCE) wb_st_a(Q[0], Q[1], Q[2], Q[3], Q[4], Q[5], G2b, cc);
    wb2_s_b(S[6], S[7], S[8], S[9], S[10], Wb, W2, H + 7);
#pragma unroll
    for (int s = 6; s < 11; ++s) Q[s] = coef * qperm(S[s]);
    Qv1 = __builtin_fma(coef, qperm(Gv), l1);
    Q2[0] = breal(0.0);
    Q2[1] = breal(0.0);
    Qv2 = l2;
    {
      const breal sc[6] = {S[6], S[7], S[8], S[9], S[10], Gv};
      sb_odd7_6(Q[6], Q[7], Q[8], Q[9], Q[10], Qv1, sc, Wo);
      const breal s2[3] = {S[9], S[10], Gv};
      sb_odd7_3(Q2[0], Q2[1], Qv2, s2, W2);
    }
    if (STANCE) {
      wb2_st_b(Q[6], Q[7], Q[8], Q[9], Q[10], Q2[0], Q2[1], G2b, G22, cc, cc2);
      Qv1 = (Qv1 + G2o[0] * ly[0]) + G2o[1] * ly[1];
      Qv2 = (Qv2 + G22[0] * ly[0]) + G22[1] * ly[1];
    }

    // ---- Qxx transpose: each row writes its half of the row rho ----
#pragma unroll
    for (int s = 0; s < 7; ++s) rl.M[at(rho, wo + s)] = Q[s];
    atomicAdd(&rl.M[at(rho, xl ? mcol(rho) : rho)], dg2);
    wave_lds_order();
    breal T[7];
    {
      lds_creal* tq = (lds_creal*)&rl.M[at(jr, cr)];
#pragma unroll
      for (int s = 0; s < 7; ++s) T[s] = lds_single(tq, at(s, 0));
    }
    wave_lds_order();

    // ---- the control block on every lane (both rows alike) ----
    wk q[4][4], Qu[4];
    q[0][0] = rbc<14>(Q[7]); q[0][1] = rbc<14>(Q[8]); q[0][2] = rbc<14>(Q[9]); q[0][3] = rbc<14>(Q[10]);
    q[1][1] = rbc<15>(Q[8]); q[1][2] = rbc<15>(Q[9]); q[1][3] = rbc<15>(Q[10]);
    q[2][2] = rbc<14>(Q2[0]); q[2][3] = rbc<14>(Q2[1]); q[3][3] = rbc<15>(Q2[1]);
    Qu[0] = rbc<14>(Qv1); Qu[1] = rbc<15>(Qv1); Qu[2] = rbc<14>(Qv2); Qu[3] = rbc<15>(Qv2);
#pragma unroll
    for (int a = 0; a < 4; ++a) q[a][a] = q[a][a] + wk(luu[a] + rc.reg);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < a; ++c) q[a][c] = q[c][a];
    bool psd;
    const Ldl4<wk> F = control_factor<wk>(q, sp.eps9, t, psd);
    wk du[4], dv = wk(0.0);
    F.neg_solve(Qu, du);
#pragma unroll
    for (int a = 0; a < 4; ++a) dv += Qu[a] * du[a];
    wk Qxu[4], K[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) Qxu[m] = wk(Q[7 + m]);
    F.neg_solve(Qxu, K);
    wk Gn = wk(Qv1);
#pragma unroll
    for (int a = 0; a < 4; ++a) Gn += K[a] * Qu[a];
    // H columns of the row: Qux[a][7 + s] lives on lane 2 s + 1; row B moves it to lane 2 s
    wk QxuS[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) QxuS[m] = qshift_rowB(Qxu[m]);
    wk Hn[7];
#pragma unroll
    for (int s = 0; s < 7; ++s) Hn[s] = wk((Q[s] + T[s]) / 2);
    wb_h_a(Hn[0], Hn[1], Hn[2], Hn[3], Hn[4], Hn[5], Hn[6], QxuS, K);
    // both rows get both halves
#pragma unroll
    for (int s = 0; s < 7; ++s) row_pair_swap(breal(Hn[s]), H[s], H[7 + s]);
    Gv = breal(Gn);
    const bool ok = gate && psd;
    pend.ok = ok && rp == 0;
    pend.k = k;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      pend.K[a] = breal(K[a]);
      pend.du[a] = breal(du[a]);
    }
    pend.G = breal(Gn);
    if (ok) rc.dV += acc(dv);
    rc.failed = rc.failed || (gate && !psd);
    if (!any_go(rc)) break;
  }
  store_pending();
  __syncthreads();
  if (xl && rp == 0) {
#pragma unroll
    for (int j = 0; j < 14; ++j) rl.M[at(rho, j)] = H[j];
    rl.Gs[rho] = Gv;
  }
  __syncthreads();
  return BWS_ITERS(it);
}

// SRB Jacobian entry of row 3+r, column col of [A B] (FBDynamics_par.c operation order).
__device__ __forceinline__ breal srb_w_entry(int r, int col, const breal* x, const breal* u,
                                              const breal* p, const breal* s, breal dt) {
  MHPC_NO_FMA
  const int row = 3 + r;
  breal ac = breal(0.0);
  if (col < 6) {
    if (row == 5 && col == 0) ac = s[0] * (kSrbInvInertia * u[1]) + s[1] * (kSrbInvInertia * u[3]);
    if (row == 5 && col == 1) ac = -(s[0] * (kSrbInvInertia * u[0]) + s[1] * (kSrbInvInertia * u[2]));
    return (col == row ? breal(1.0) : breal(0.0)) + ac * dt;
  }
  const int c = col - 6;
  breal bc = breal(0.0);
  if (row == 3 && c == 0) bc = kSrbInvMass * s[0];
  if (row == 5 && c == 0) bc = s[0] * (kSrbInvInertia * (p[1] - x[1]));
  if (row == 4 && c == 1) bc = kSrbInvMass * s[0];
  if (row == 5 && c == 1) bc = -(s[0] * (kSrbInvInertia * (p[0] - x[0])));
  if (row == 3 && c == 2) bc = kSrbInvMass * s[1];
  if (row == 5 && c == 2) bc = s[1] * (kSrbInvInertia * (p[3] - x[1]));
  if (row == 4 && c == 3) bc = kSrbInvMass * s[1];
  if (row == 5 && c == 3) bc = -(s[1] * (kSrbInvInertia * (p[2] - x[0])));
  return bc * dt;
}

// Row 5 (theta) of W, column col, from the lane's two knot operands (srb_w_entry(2, ...) term
// for term): e0, e1 = u1, u3 (col 0) / u0, u2 (col 1); e0 = z (cols 6, 8) / x (cols 7, 9).
__device__ __forceinline__ breal srb_w2_lane(int col, breal e0, breal e1, const breal* p, const breal* s,
                                            breal dt) {
  MHPC_NO_FMA
  // every candidate term, then selects (no divergent branches in the knot loop)
  const int c = col - 6;
  // (values first, then selects: a select between addresses of the caller's array would
  // keep that array in scratch)
  const breal f0 = p[0], f1 = p[1], f2 = p[2], f3 = p[3], s0 = s[0], s1 = s[1];
  breal pp = f2;
  pp = c == 2 ? f3 : pp;
  pp = c == 1 ? f0 : pp;
  pp = c == 0 ? f1 : pp;
  const breal bs = (c < 2 ? s0 : s1) * (kSrbInvInertia * (pp - e0));
  const breal ia = s0 * (kSrbInvInertia * e0) + s1 * (kSrbInvInertia * e1);
  const breal ac = col == 0 ? ia : col == 1 ? -ia : breal(0.0);
  const breal bc = (c & 1) ? -bs : bs;
  return col < 6 ? (col == 5 ? breal(1.0) : breal(0.0)) + ac * dt : bc * dt;
}
// Knot-record offsets of a lane's two W-row-5 operands (see srb_w2_lane)
__device__ __forceinline__ int srb_w2_off(int col, int which) {
  if (col == 0) return which ? 9 : 7;  // u3 : u1
  if (col == 1) return which ? 8 : 6;  // u2 : u0
  if (which == 0 && col >= 6) return (col & 1) ? 0 : 1;  // x (cols 7, 9) : z (cols 6, 8)
  return 0;  // unused
}

// Operand prefetch distance of the SRB half's sweep in knots (1: the next knot's operands load
// while the current one computes; 2: two knots ahead, in two alternating register sets).  2
// measured -4 % per SRB-half launch at batch 1024 and -13 % at 4096 (beside the partials, whose
// traffic lengthens the loads' round trips) but does not fit the half's 256-VGPR budget (a few
// loop-invariant values go to scratch, which the build gate refuses), so 1
#ifndef MHPC_BWS_SRB_PF
#define MHPC_BWS_SRB_PF 1
#endif
constexpr int SRB_PF_HALF = MHPC_BWS_SRB_PF;

// ---------------------------------------------------------------------------------------
// SRB phase (NQ = 3): the Jacobians are evaluated in registers (FBDynamics_par.c), the cost
// derivatives from the nominal knot (CostBase.cpp:19-34).
// LANE_OPS: each lane loads only its row-5 operands (srb_w2_lane); otherwise x, z and u (the
// whole-sweep kernels: their register allocation is the WB knots', measured slower with it)
template <int SRB_PF, bool LANE_OPS>
__device__ int sweep_srb(const SolveParams& sp, const DevBufs& d, const Layout& L, const ProbState* st, RowLds& rl,
                          RowCtx& rc, int p) {
  using R = Rows<3>;
  const int t = rc.t, b = rc.b;
  const int N = L.N[p], ko = L.ko[p], mode = L.mode[p];
  const breal dt = L.dt[p];
  const int rho = R::rho(t);
  const bool xl = t < 6;
  const int cj = rho < 10 ? rho : 0;  // column of [A B] held (clamped for spare lanes)
  const breal coef = xl ? ((t & 1) ? dt : breal(1.0)) : breal(0.0);
  // foothold and contact flags in the model's type, as the line search planned them
  breal foot[4], cs[2];
  {
    real fr[4], cr2[2];
    plan_foothold(traj_ptr(sp, d, b, rc.nom, ko), L.dt[p] * N, mode, fr);
    srb_contact(mode, cr2);
#pragma unroll
    for (int i = 0; i < 4; ++i) foot[i] = fr[i];
    cs[0] = cr2[0];
    cs[1] = cr2[1];
  }
  const int m = mode - 1;
  // per-lane cost weight 2 dt Q / 2 dt R and fixed reference of row cj
  breal w2, rxc;
  if (cj < 6) {
    w2 = 2 * dt * sp.cw.fQ[m][cj];
    rxc = cj == 1 ? sp.height : cj == 3 ? sp.vel : breal(0.0);
  } else {
    const int c = cj - 6;
    w2 = 2 * dt * sp.cw.fR[m][c];
    rxc = (c == 1 || c == 3) ? breal(8.252) * breal(9.81) : breal(0.0);
  }
  breal luu[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) luu[c] = 2 * dt * sp.cw.fR[m][c];
  // lxx + reg, see sweep_wb (two-row layout: both rows run this phase, row A adds)
  const breal dg2 = xl && rc.rp == 0 ? 2 * (w2 + rc.reg) : breal(0.0);
  // rows 3, 4 of W do not depend on the knot
  const breal zx[2] = {0, 0}, zu[4] = {0, 0, 0, 0};
  const breal W0c = srb_w_entry(0, cj, zx, zu, foot, cs, dt);
  const breal W1c = srb_w_entry(1, cj, zx, zu, foot, cs, dt);
  const real* pos = d.refpos + (size_t)b * sp.NK + ko;
  // a lane's knot operands from the nominal: its two W-row-5 operands (or x, z, u), its own
  // entry, the position reference
  struct Ops {
    real e0, e1, v, pos, xs[2], us[4];  // record type, see sweep_wb
  };
  const real* tk0 = traj_ptr(sp, d, b, rc.nom, ko);  // knot k adds k KS
  const int oe0 = srb_w2_off(cj, 0), oe1 = srb_w2_off(cj, 1);
  auto load = [&](int k, Ops& o) __attribute__((always_inline)) {
    const real* tk = tk0 + k * KS;
    o.pos = pos[k];
    o.v = tk[cj];
    if (LANE_OPS) {
      o.e0 = tk[oe0];
      o.e1 = tk[oe1];
    } else {
      o.xs[0] = tk[0]; o.xs[1] = tk[1];
#pragma unroll
      for (int c = 0; c < 4; ++c) o.us[c] = tk[6 + c];
    }
  };
  breal H[6], Gv;
  {
    const int hr = xl ? rho : 0;
#pragma unroll
    for (int j = 0; j < 6; ++j) H[j] = rl.M[at(hr, j)];
    Gv = rl.Gs[hr];
  }
  const int cr = rho < 10 ? rho : 0;
  PendingKnot pend;  // outputs stored one knot later (see sweep_wb)
  pend.ok = false;
  const size_t rec0 = (size_t)b * sp.NK + ko;
  real* const K0 = d.K + rec0 * 56 + rho;
  real* const G0 = d.G + rec0 * 14 + rho;
  real* const du0 = d.du + rec0 * 4;
  auto store_pending = [&]() {
    if (pend.ok) {
      if (xl) {
#pragma unroll
        for (int a = 0; a < 4; ++a) K0[pend.k * 56 + a * 6] = pend.K[a];
        G0[pend.k * 14] = pend.G;
      } else if (t == 6) {
#pragma unroll
        for (int a = 0; a < 4; ++a) du0[pend.k * 4 + a] = pend.du[a];
      }
    }
    pend.ok = false;
  };
  Ops oa, ob;
#ifdef MHPC_BWS_TIMING
  unsigned long long segacc[5] = {0, 0, 0, 0, 0};
#endif
  if (N >= 2) load(N - 2, oa);
  if (SRB_PF > 1 && N >= 3) load(N - 3, ob);
  int it = 0;  // knot iterations the wave ran (the cycle accounting's knot count)
  // knot k from operand set o; refills o with the operands of knot k - SRB_PF.  False: no row
  // of the wave goes on
  auto knot = [&](int k, Ops& o) __attribute__((always_inline)) {
    ++it;
    BWS_T(sg0);
    breal W[3];
    W[0] = W0c;
    W[1] = W1c;
    if (LANE_OPS) {
      W[2] = srb_w2_lane(cj, breal(o.e0), breal(o.e1), foot, cs, dt);
    } else {
      const breal xs[2] = {o.xs[0], o.xs[1]}, us[4] = {o.us[0], o.us[1], o.us[2], o.us[3]};
      W[2] = srb_w_entry(2, cj, xs, us, foot, cs, dt);
    }
    const breal rxi = rho == 0 ? breal(o.pos) : rxc;
    const breal l1 = w2 * (breal(o.v) - rxi);
    const bool gate = go(rc);
    rc.kn += gate ? 1 : 0;
    asm volatile("" ::"v"(W[2]), "v"(l1));  // see sweep_wb
    // (distance 2: issued ahead of the knot's stores, so that the wait for it -- gfx950's single
    // in-order VM counter -- covers no store of the knot before its use)
    if (SRB_PF > 1 && k >= SRB_PF) load(k - SRB_PF, o);
    store_pending();
    if (SRB_PF == 1 && k > 0) load(k - 1, o);
    BWS_SEG(8, sg0, sg1);
    breal S[10];
#pragma unroll
    for (int c = 0; c < 3; ++c) S[c] = H[c];
#pragma unroll
    for (int c = 3; c < 6; ++c) S[c] = dt * H[c - 3];
#pragma unroll
    for (int c = 6; c < 10; ++c) S[c] = breal(0.0);
    // (only the structurally non-zero W terms: W is 5 + 8 non-zeros, FBDynamics_par.c:53-54)
    srb_sp_a(S[0], S[1], S[3], S[4], W, H + 3);
    breal Q[10], Qv1;
#pragma unroll
    for (int c = 0; c < 5; ++c) Q[c] = coef * qperm(S[c]);
    sb_odd3_5(Q[0], Q[1], Q[2], Q[3], Q[4], S + 0, W);
    srb_sp_b(S[5], S[6], S[7], S[8], S[9], W, H + 3);
#pragma unroll
    for (int c = 5; c < 10; ++c) Q[c] = coef * qperm(S[c]);
    Qv1 = __builtin_fma(coef, qperm(Gv), l1);
    {
      const breal sc[6] = {S[5], S[6], S[7], S[8], S[9], Gv};
      sb_odd3_6(Q[5], Q[6], Q[7], Q[8], Q[9], Qv1, sc, W);
    }
    BWS_SEG(9, sg1, sg2);
#pragma unroll
    for (int j = 0; j < 10; ++j) rl.M[at(rho & 15, j)] = Q[j];
    atomicAdd(&rl.M[at(rho & 15, rho & 15)], dg2);  // see sweep_wb
    wave_lds_order();
    breal T[6];
    {
      lds_creal* tq = (lds_creal*)&rl.M[at(0, cr)];
#pragma unroll
      for (int j = 0; j < 6; ++j) T[j] = lds_single(tq, at(j, 0));
    }
    wave_lds_order();
    BWS_SEG(10, sg2, sg3);
    breal q[4][4], Qu[4];
    q[0][0] = rbc<6>(Q[6]); q[0][1] = rbc<6>(Q[7]); q[0][2] = rbc<6>(Q[8]); q[0][3] = rbc<6>(Q[9]);
    q[1][1] = rbc<7>(Q[7]); q[1][2] = rbc<7>(Q[8]); q[1][3] = rbc<7>(Q[9]);
    q[2][2] = rbc<8>(Q[8]); q[2][3] = rbc<8>(Q[9]); q[3][3] = rbc<9>(Q[9]);
    Qu[0] = rbc<6>(Qv1); Qu[1] = rbc<7>(Qv1); Qu[2] = rbc<8>(Qv1); Qu[3] = rbc<9>(Qv1);
#pragma unroll
    for (int a = 0; a < 4; ++a) q[a][a] = q[a][a] + (luu[a] + rc.reg);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < a; ++c) q[a][c] = q[c][a];
    bool psd;
    const Ldl4<breal> F = control_factor<breal>(q, sp.eps9, t, psd);
    breal du[4], dv = breal(0.0);
    F.neg_solve(Qu, du);
#pragma unroll
    for (int a = 0; a < 4; ++a) dv += Qu[a] * du[a];
    breal Qxu[4], K[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) Qxu[c] = Q[6 + c];
    F.neg_solve(Qxu, K);
    breal Gn = Qv1;
#pragma unroll
    for (int a = 0; a < 4; ++a) Gn += K[a] * Qu[a];
    BWS_SEG(11, sg3, sg4);
    breal Hn[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) Hn[j] = (Q[j] + T[j]) / 2;
    srb_h(Hn[0], Hn[1], Hn[2], Hn[3], Hn[4], Hn[5], Qxu, K);
#pragma unroll
    for (int j = 0; j < 6; ++j) H[j] = Hn[j];
    Gv = Gn;
    const bool ok = gate && psd;
    pend.ok = ok && rc.rp == 0;
    pend.k = k;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      pend.K[a] = K[a];
      pend.du[a] = du[a];
    }
    pend.G = Gn;
    if (ok) rc.dV += acc(dv);
    rc.failed = rc.failed || (gate && !psd);
    const bool more = any_go(rc);
    BWS_SEG(12, sg4, sg5);
    return more;
  };
  if (SRB_PF == 1) {
    for (int k = N - 2; k >= 0; --k)
      if (!knot(k, oa)) break;
  } else {
    // sets alternate (no register copies: a copy would wait for the load on the spot)
    for (int k = N - 2; k >= 0; k -= 2) {
      if (!knot(k, oa) || k == 0) break;
      if (!knot(k - 1, ob)) break;
    }
  }
  store_pending();
#ifdef MHPC_BWS_TIMING
  for (int i = 0; i < 5; ++i) BWS_ADD(8 + i, segacc[i]);
#endif
  __syncthreads();
  if (xl) {
#pragma unroll
    for (int j = 0; j < 6; ++j) rl.M[at(rho, j)] = H[j];
    rl.Gs[rho] = Gv;
  }
  __syncthreads();
  return BWS_ITERS(it);
}

// ---------------------------------------------------------------------------------------
// Terminal value function of phase p (SinglePhase.cpp:189-191) in LDS: G = Phix + Gnext,
// H = Phixx + Hnext; AL partials only while st->al_partials (quirk B1).  G of knot N-1 is
// an output of the phase.
template <int NX>
__device__ void terminal_value(const SolveParams& sp, const DevBufs& d, const Layout& L, const ProbState* st,
                               RowLds& rl, const RowCtx& rc, int p) {
  constexpr bool wb = NX == 14;
  const int mode = L.mode[p], N = L.N[p], ko = L.ko[p];
  const breal pos = d.refpos[(size_t)rc.b * sp.NK + ko + N - 1];
  const real* xe = traj_ptr(sp, d, rc.b, rc.nom, ko + N - 1);
  const bool al = wb && ntc_of(mode, true) && sp.AL_active && st->al_partials;
  if (al && rc.lt == 0) {
    real hx[14], Hs[3][3], h;  // (the model's type)
    if (mode == 2) wb_touchdown_compact<kFront>(xe, &h, hx, Hs);
    else wb_touchdown_compact<kBack>(xe, &h, hx, Hs);
#pragma unroll
    for (int i = 0; i < 14; ++i) rl.hx[i] = hx[i];
#pragma unroll
    for (int i = 0; i < 9; ++i) rl.Hs[i] = Hs[i / 3][i % 3];
    rl.h = h;
  }
  __syncthreads();
  const breal h = al ? rl.h : breal(0.0);
  const breal s = st->sigma[p], lam = st->lambda[p];
  const int ih = mode == 2 ? 3 : 5;  // touchdown Hessian block (theta, hip, knee)
  real* Gout = d.G + ((size_t)rc.b * sp.NK + ko + N - 1) * 14;
  const bool gate = go(rc);
  #pragma unroll 1
  for (int e = rc.lt; e < NX * NX + NX; e += rc.nl) {
    if (e < NX * NX) {
      const int i = e / NX, j = e - i * NX;
      breal v = i == j ? (wb ? sp.cw.wQf[mode - 1][i] : sp.cw.fQf[mode - 1][i]) : breal(0.0);
      if (al) {
        const int ai = i == 2 ? 0 : (i == ih ? 1 : (i == ih + 1 ? 2 : -1));
        const int aj = j == 2 ? 0 : (j == ih ? 1 : (j == ih + 1 ? 2 : -1));
        const breal hij = (ai >= 0 && aj >= 0) ? rl.Hs[ai * 3 + aj] : breal(0.0);
        v += 50 * (s * s / 2 * (rl.hx[i] * rl.hx[j] + h * hij) + lam * hij);
      }
      rl.M[at(i, j)] = v + rl.M[at(i, j)];
    } else {
      const int i = e - NX * NX;
      breal rxi;
      if (wb) rxi = i == 0 ? pos : (i == 7 ? sp.vel : cXtermWB[mode - 1][i]);
      else rxi = i == 0 ? pos : (i == 1 ? sp.height : (i == 3 ? sp.vel : breal(0.0)));
      breal v = (wb ? sp.cw.wQf[mode - 1][i] : sp.cw.fQf[mode - 1][i]) * (xe[i] - rxi);
      if (al) v += 50 * (s * s / 2 * rl.hx[i] * h + lam * rl.hx[i]);
      const breal g = v + rl.Gs[i];
      rl.Gs[i] = g;
      if (gate) Gout[i] = g;
    }
  }
  __syncthreads();
}

// impact_aware_step (MultiPhaseDDP.cpp:300-341) for a WB phase p: rl.M / rl.Gs hold CTG[0] of
// phase p+1 (6-dim if that phase is SRB); on exit the 14-dim Gnext / Hnext of phase p.
__device__ void impact_step(const SolveParams& sp, const DevBufs& d, const Layout& L, RowLds& rl, RowCtx& rc, int p) {
  using R = Rows<7>;
  const int t = rc.t;
  const int mode = L.mode[p];
  const bool nwb = p + 1 < L.n_wb;
  const bool imp = mode == 2 || mode == 4;
  const int i = t < 14 ? R::rho(t) : 0;
  // lift to the full-model space: E' G', E' H' E (E = _stateProj for an SRB next phase)
  breal H2[14], G2v;
  {
    const int pi = nwb ? i : (i < 3 ? i : (i >= 7 && i < 10 ? i - 4 : -1));
    const int pr = pi >= 0 ? pi : 0;
#pragma unroll
    for (int j = 0; j < 14; ++j) {
      const int pj = nwb ? j : (j < 3 ? j : (j >= 7 && j < 10 ? j - 4 : -1));
      const breal v = pj >= 0 ? rl.M[at(pr, pj)] : breal(0.0);
      H2[j] = pi >= 0 ? v : breal(0.0);
    }
    G2v = pi >= 0 ? rl.Gs[pr] : breal(0.0);
  }
  breal Hn[14], Gn;
  if (imp) {
    // Px column i (column-major record): Pc[m] = Px[m][i]
    const real* pxc = d.px + ((size_t)rc.b * MAXP + p) * 196 + i * 14;
    breal Pc[14];
#pragma unroll
    for (int m = 0; m < 14; ++m) Pc[m] = pxc[m];
    if (go(rc) && t == 0) ++rc.px_reads;
    // T = Px' H2 (lane: row i), G = Px' G2: sum over m = 0..13 in order
    breal T[14];
#pragma unroll
    for (int j = 0; j < 14; ++j) T[j] = breal(0.0);
    Gn = breal(0.0);
    {
      const breal h2b[8] = {H2[7], H2[8], H2[9], H2[10], H2[11], H2[12], H2[13], G2v};
      sb_even7_7(T[0], T[1], T[2], T[3], T[4], T[5], T[6], H2, Pc);
      sb_even7_8(T[7], T[8], T[9], T[10], T[11], T[12], T[13], Gn, h2b, Pc);
      sb_odd7_7(T[0], T[1], T[2], T[3], T[4], T[5], T[6], H2, Pc + 7);
      sb_odd7_8(T[7], T[8], T[9], T[10], T[11], T[12], T[13], Gn, h2b, Pc + 7);
    }
    // H = T Px: H[i][j] = sum_m T[i][m] Px[m][j], Px[m][j] on lane lam(j)
#pragma unroll
    for (int j = 0; j < 14; ++j) Hn[j] = breal(0.0);
    wb_p_a(Hn[0], Hn[1], Hn[2], Hn[3], Hn[4], Hn[5], Hn[6], Pc, T);
    wb_p_b(Hn[7], Hn[8], Hn[9], Hn[10], Hn[11], Hn[12], Hn[13], Pc, T);
    wb_p_a(Hn[0], Hn[1], Hn[2], Hn[3], Hn[4], Hn[5], Hn[6], Pc + 7, T + 7);
    wb_p_b(Hn[7], Hn[8], Hn[9], Hn[10], Hn[11], Hn[12], Hn[13], Pc + 7, T + 7);
  } else {
#pragma unroll
    for (int j = 0; j < 14; ++j) Hn[j] = H2[j];
    Gn = G2v;
  }
  __syncthreads();
  if (t < 14) {
#pragma unroll
    for (int j = 0; j < 14; ++j) rl.M[at(i, j)] = Hn[j];
    rl.Gs[i] = Gn;
  }
  __syncthreads();
}


// One sweep attempt over phases p_hi..p_lo (MultiPhaseDDP::backward_sweep).  On entry
// rl.M / rl.Gs hold the value function entering phase p_hi (zero for the last phase) and
// rc.dV the matching dVnext.
// WB_CODE = false: SRB phases only (the SRB half of a split sweep), no whole-body code in the
// kernel (its register allocation is the SRB knot's, so a partials wave fits beside it).
// RPP: rows per problem (2: the whole-body phases run sweep_wb2, SRB phases on both rows).
template <bool WB_CODE, int RPP>
__device__ void sweep_phases(const SolveParams& sp, const DevBufs& d, const Layout& L, ProbState* st, RowLds& rl,
                             RowCtx& rc, int p_hi, int p_lo) {
  for (int p = p_hi; p >= p_lo; --p) {
    const bool wb = WB_CODE && p < L.n_wb;
    const bool was_go = go(rc);
    if (p + 1 < L.P) {
      if constexpr (WB_CODE) {
        BWS_T(ti0);
        if (wb) impact_step(sp, d, L, rl, rc, p);
        BWS_ADD(5, clock64() - ti0);
      }
      if (was_go) rc.dV = st->dV[p + 1];  // dVnext
    }
    BWS_T(tt0);
    if (wb) {
      if constexpr (WB_CODE) {
        terminal_value<14>(sp, d, L, st, rl, rc, p);
        BWS_ADD(4, clock64() - tt0);
        BWS_T(tw0);
        const int mode = L.mode[p];
        int nit;
        if (RPP == 2) {
          if (mode == 1 || mode == 3) nit = sweep_wb2<true>(sp, d, L, st, rl, rc, p);
          else nit = sweep_wb2<false>(sp, d, L, st, rl, rc, p);
        } else {
          if (mode == 1 || mode == 3) nit = sweep_wb<true>(sp, d, L, st, rl, rc, p);
          else nit = sweep_wb<false>(sp, d, L, st, rl, rc, p);
        }
        BWS_ADD(0, clock64() - tw0);
        BWS_ADD(1, nit);
        (void)nit;
      }
    } else {
      terminal_value<6>(sp, d, L, st, rl, rc, p);
      BWS_ADD(4, clock64() - tt0);
      BWS_T(ts0);
      // (the whole-sweep kernels keep distance 1 and x, z, u operands: their registers go to
      // the WB knots)
      const int nit = sweep_srb<WB_CODE ? 1 : SRB_PF_HALF, !WB_CODE>(sp, d, L, st, rl, rc, p);
      BWS_ADD(2, clock64() - ts0);
      BWS_ADD(3, nit);
      (void)nit;
    }
    if (was_go && rc.lt == 0) st->dV[p] = rc.dV;
    if (!any_go(rc)) break;
  }
}

// Zero value function entering the last phase (MultiPhaseDDP.cpp:103-105).
__device__ void zero_value(RowLds& rl, RowCtx& rc) {
  __syncthreads();
  #pragma unroll 1
  for (int e = rc.lt; e < 16 * MP; e += rc.nl) rl.M[e] = breal(0.0);
  if (rc.lt < 16) rl.Gs[rc.lt] = breal(0.0);
  rc.dV = acc(0.0);
  __syncthreads();
}

// Waves per SIMD the register allocator leaves room for in the SRB half: it runs beside the
// partials; capped at 256 VGPRs (A/B round 4: a 168-VGPR cap that lets a 340-VGPR partials
// wave share the SIMD spills the SRB knot to scratch and loses 2 % of a batch-1024 step).
#ifndef MHPC_BWS_SRB_WAVES
#define MHPC_BWS_SRB_WAVES 2
#endif

// RPW problems per wave, RPP rows per problem (rows 0..RPW*RPP-1 of the wave; the others
// idle).  RPP = 2 (RPW = 2): problem q on rows 2q, 2q+1 sharing one RowLds (sweep_wb2).
//
// PART 0: the whole sweep with its regularisation retries (MultiPhaseDDP.cpp:196-241).
// PART 1: the SRB phases of the attempts until one passes them (an attempt that fails there
// never reaches a WB phase, so it is wholly done here: with the reference's default weights the
// first DDP iteration of every AL iteration fails its first attempt at the first knot), the
// value function at the WB boundary saved to d.carry (this launch runs beside the partials,
// which it does not read).
// PART 2: the WB phases of that attempt, then the same retries as PART 0 (whole sweeps) --
// the same attempts with the same regularisation, bit for bit.
template <int RPW, int PART, int RPP>
__global__ __launch_bounds__(64, PART == 1 ? MHPC_BWS_SRB_WAVES : 1) void k_bws(SolveParams sp, DevBufs d,
                                                                    real update_reg) {
  static_assert(RPP == 1 || (RPP == 2 && RPW == 2 && PART != 1), "row layout");
  __shared__ BwsLds sh;
  BWS_T(tk0);
  const int row = threadIdx.x >> 4;
  const int q = RPP == 2 ? row >> 1 : row;  // problem slot of the row
  RowCtx rc;
  rc.t = threadIdx.x & 15;
  rc.rp = RPP == 2 ? row & 1 : 0;
  rc.lt = rc.t + 16 * rc.rp;
  rc.nl = 16 * RPP;
  // the block's layout group and problems (a block never mixes layouts)
  const GrpBlk gb = block_group(sp, blockIdx.x, RPW);
  if (gb.g < 0) return;
  const Layout& L = layout_of(d, gb.g);
  const bool inb = q < RPW && gb.p0 + q < gb.p1;
  rc.b = prob_at(sp, d, inb ? gb.p0 + q : gb.p0);  // a spare row shadows the block's first problem
  ProbState* st = &d.st[rc.b];
  rc.act = inb && st->active && st->ddp_active;
  if (!__builtin_amdgcn_ballot_w64(rc.act)) return;
  RowLds& rl = sh.r[q];
  rc.nom = st->nom_slot;
  rc.reg = st->reg;
  rc.kn = rc.kn_wb = rc.px_reads = 0;
  rc.dV = acc(0.0);
  int bws_iter = 1;
  int64_t sweeps = 0;
  bool aborted = false;
  bool pending = rc.act;
  for (bool first = true;; first = false) {
    rc.live = pending;
    rc.failed = false;
    sweeps += rc.live ? 1 : 0;
    if (PART == 1) {
      zero_value(rl, rc);
      // (a layout without SRB phases passes with nothing swept; PART 2 sweeps it whole)
      if (L.P > L.n_wb) sweep_phases<false, 1>(sp, d, L, st, rl, rc, L.P - 1, L.n_wb);
      BwsCarry& c = d.carry[rc.b];
      __syncthreads();
      if (rc.live && !rc.failed) {  // (now: a later attempt of another row reuses rl)
        #pragma unroll 1
        for (int e = rc.t; e < 36; e += 16) c.H[e] = rl.M[at(e / 6, e % 6)];
        if (rc.t < 6) c.G[rc.t] = rl.Gs[rc.t];
      }
      pending = rc.live && rc.failed;
      if (pending) {  // the next attempt, as PART 0 would start it
        rc.reg = fmax(rc.reg * update_reg, breal(1e-03));
        ++bws_iter;
        if (rc.reg > 1000) {
          aborted = true;
          pending = false;
        }
      }
      if (__builtin_amdgcn_ballot_w64(pending)) continue;
      if (rc.act) {
        if (rc.t == 0) {
          c.reg = rc.reg;
          c.abort = aborted ? 1 : 0;
          c.iter = bws_iter;
          c.sweeps = (int32_t)sweeps;
          c.knots = (int32_t)rc.kn;
        }
      }
      return;
    }
    if (PART == 2 && first && L.P > L.n_wb) {
      // resume the SRB half's passing attempt from its value function (its regularisation,
      // its attempt number) -- or take over its abort
      const BwsCarry& c = d.carry[rc.b];
      __syncthreads();
      #pragma unroll 1
      for (int e = rc.lt; e < 36; e += rc.nl) rl.M[at(e / 6, e % 6)] = c.H[e];
      if (rc.lt < 6) rl.Gs[rc.lt] = c.G[rc.lt];
      __syncthreads();
      if (rc.live) {
        rc.reg = c.reg;
        bws_iter = c.iter;
        sweeps += c.sweeps - 1;
        rc.kn += c.knots;
        aborted = c.abort != 0;
      }
      rc.failed = rc.live && aborted;
      rc.dV = st->dV[L.n_wb];
      sweep_phases<true, RPP>(sp, d, L, st, rl, rc, L.n_wb - 1, 0);
    } else {
      zero_value(rl, rc);
      sweep_phases<true, RPP>(sp, d, L, st, rl, rc, L.P - 1, 0);
    }
    pending = rc.live && rc.failed && !aborted;
    if (pending) {
      rc.reg = fmax(rc.reg * update_reg, breal(1e-03));  // MultiPhaseDDP.cpp:218
      ++bws_iter;
      if (rc.reg > 1000) {
        aborted = true;
        pending = false;
      }
    }
    if (!__builtin_amdgcn_ballot_w64(pending)) break;
  }
  BWS_ADD(6, clock64() - tk0);
  BWS_ADD(7, 1);
  if (rc.act && rc.lt == 0) {
    st->cnt[C_DDP]++;
    st->cnt[C_BWS] += sweeps;
    st->cnt[C_BWS_KNOTS] += rc.kn;
    st->cnt[C_BWS_KNOTS_WB] += rc.kn_wb;
    st->cnt[C_BWS_KNOTS_FB] += rc.kn - rc.kn_wb;
    st->cnt[C_PX_READS] += rc.px_reads;
    if (PART == 2) st->cnt[C_BWS_KNOTS_FB1] += d.carry[rc.b].knots;
    st->bws_iter = bws_iter;
    if (aborted) {  // "Regularization term exceeds maximum value": return from solve()
      st->status = MHPC_SOLVE_REG_ABORT;
      st->active = 0;
      st->ddp_active = 0;
      if (st->ntrace < TRACE)
        st->trace[st->ntrace++] = (st->al_iter << 24) | (st->reb_active << 23) | (1 << 21) |
                                  (bws_iter & 0xff);
    } else {
      st->dV_exp = st->dV[0];  // _exp_cost_change = _phases[0]->_dV
      breal reg = rc.reg / 20;  // MultiPhaseDDP.cpp:237-241
      if (reg < breal(1e-06)) reg = 0;
      st->reg = reg;
    }
  }
}

// Launch shape: sp.var_bws (mhpc_set_kernel_variant) or bws_auto_variant.  Two / one
// problems per wave run the same per-row code on fewer rows; PAIRS2 runs the whole-body phases
// on two rows per problem (tests/test_gpu_variants.py checks them all bit for bit).
// part: 0 whole sweep, 1 / 2 its SRB / WB halves (bws_split).
// Default shape: one row per problem (four per wave) fills the chip from about a thousand
// problems; up to 2048 the two-row layout (half the whole-body knot per row) is faster.
#ifndef MHPC_BWS_PAIRS_MAX_B
#define MHPC_BWS_PAIRS_MAX_B 2048
#endif
// Blocks of `rpw` problems over the layout groups (block_group)
static unsigned bws_grid(const SolveParams& sp, int rpw) {
  long n = 0;
  for (int g = 0; g < sp.ngrp; ++g) n += (sp.go[g + 1] - sp.go[g] + rpw - 1) / rpw;
  return (unsigned)n;
}
int bws_auto_variant(int B) {
  return B <= MHPC_BWS_PAIRS_MAX_B ? MHPC_VARIANT_BWS_PAIRS2 : MHPC_VARIANT_BWS_ROWS4;
}

hipError_t launch_bws(const SolveParams& sp, const DevBufs& d, real update_reg, int part,
                      hipStream_t s) {
  const int v = sp.var_bws ? sp.var_bws : bws_auto_variant(launch_problems(sp));
  const int rpw = v == MHPC_VARIANT_BWS_ROWS1 ? 1 : (v == MHPC_VARIANT_BWS_ROWS2 ||
                                                     v == MHPC_VARIANT_BWS_PAIRS2) ? 2 : 4;
  const dim3 grid(bws_grid(sp, rpw));
  const dim3 grid4(bws_grid(sp, 4));
#define MHPC_LAUNCH_BWS(R)                                                                    \
  do {                                                                                        \
    if (part == 1) hipLaunchKernelGGL((k_bws<R, 1, 1>), grid, dim3(64), 0, s, sp, d, update_reg); \
    else if (part == 2) hipLaunchKernelGGL((k_bws<R, 2, 1>), grid, dim3(64), 0, s, sp, d, update_reg); \
    else hipLaunchKernelGGL((k_bws<R, 0, 1>), grid, dim3(64), 0, s, sp, d, update_reg);           \
  } while (0)
  if (v == MHPC_VARIANT_BWS_PAIRS2) {
    // the SRB half keeps one row per problem (its knot is short; four problems per wave)
    if (part == 1) hipLaunchKernelGGL((k_bws<4, 1, 1>), grid4, dim3(64), 0, s, sp, d, update_reg);
    else if (part == 2) hipLaunchKernelGGL((k_bws<2, 2, 2>), grid, dim3(64), 0, s, sp, d, update_reg);
    else hipLaunchKernelGGL((k_bws<2, 0, 2>), grid, dim3(64), 0, s, sp, d, update_reg);
  } else if (rpw == 1) MHPC_LAUNCH_BWS(1);
  else if (rpw == 2) MHPC_LAUNCH_BWS(2);
  else MHPC_LAUNCH_BWS(4);
#undef MHPC_LAUNCH_BWS
  return hipGetLastError();
}

// Whether the sweep runs as an SRB launch beside the partials and a WB launch after them:
// both kinds of phase present, not switched off (var_overlap 2).
bool bws_split(const SolveParams& sp) {
  return sp.split_ok && sp.var_overlap != 2;
}

#ifdef MHPC_BWS_VARIANT_NS
}  // namespace MHPC_BWS_VARIANT_NS
#endif
}  // namespace MHPC_NS

#ifdef MHPC_BWS_TIMING
extern "C" int mhpc_dbg_bws_cycles(unsigned long long* out, int reset) {
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(MHPC_NS::g_bws_cyc), sizeof(unsigned long long) * 16) !=
      hipSuccess)
    return 1;
  if (reset) {
    unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(MHPC_NS::g_bws_cyc), z, sizeof(z)) != hipSuccess) return 1;
  }
  return 0;
}
#endif
