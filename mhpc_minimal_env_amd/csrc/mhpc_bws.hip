// k_bws: the backward Riccati sweep of the batched HSDDP solve, one wavefront per problem.
//
// Restates MultiPhaseDDP::backward_sweep + impact_aware_step (MultiPhaseDDP.cpp:100-127,
// 300-341), SinglePhase::backward_sweep (SinglePhase.cpp:183-216), compute_Qfunction and
// valuefunction_update (MHPC_CompoundTypes.h:117-144) and the regularisation retry loop of
// MultiPhaseDDP::solve (:196-241).
//
// Per knot the 64 lanes share the dense blocks through LDS.  The dynamics Jacobian of a
// planar model with state (q, qdot) and explicit Euler always has the shape
//     [A B] = [ I  dt*I  0 ]      (rows 0..NQ-1, exact)
//             [    W       ]      (rows NQ..NX-1: W = rows of I + dt*Ac | dt*Bc)
// so every product with A or B is  a(col) * M[.., b(col)] + sum_r M[.., NQ+r] * W[r][col]
// with a = 1 / dt / 0 and b = col / col-NQ.  Skipping the structural zeros of the dense
// products of the reference changes no rounding (the skipped terms are exact zeros and the
// remaining terms are summed in the same order).  C and D are non-zero only in the two
// force rows of the stance foot (G2), and so is lyy.
//
// Knot pipeline: the partials record of knot k-1 and its nominal state are loaded into
// registers while knot k computes, and dropped into LDS at the top of the next knot.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "mhpc_device.h"

namespace MHPC_NS {

// Padded LDS shapes: every lane of a round runs the same straight-line code; rows / columns
// past the real extents land in padding that no real output reads.
// Sized for the 64- and the 128-thread block (see riccati_knot's static_asserts).
constexpr int WS = 24;          // row stride of W / G2 (columns of [A B], padded)
constexpr int JR = 24;          // rows of Jt (padded)
constexpr int QR = 24;          // rows of Q (padded)
// Row stride of Jt: NX + 1 puts the rows a half-wave reads together in R3 on distinct LDS
// banks (stride NX = 14 doubles maps rows 16, 17 onto the banks of rows 0, 1).
#ifndef MHPC_BWS_JTPAD
#define MHPC_BWS_JTPAD 1
#endif
// Column-major blocks (MHPC_BWS_WT=1, default): the NQ dynamic rows of one column of [A B]
// are contiguous in W (stride WR), the two stance rows of one column of [C D] in G2, and
// the NQ entries Jt[row][NQ..NX-1] that R3 keeps in registers start 16-byte aligned (one
// leading pad element per row), so R2 and R3 read their operand runs with ds_read_b128
// (4 LDS cycles for 16 bytes per lane) instead of strided ds_read2_b64 pairs (8 cycles).
// Jt row strides 18 / 10 doubles put the rows of a 16-lane b128 group on distinct banks
// (tools/lds_bank_model_r3.py).  Only the LDS layout changes: same products, same order.
#ifndef MHPC_BWS_WT
#define MHPC_BWS_WT 1
#endif
#ifndef MHPC_BWS_WR
#define MHPC_BWS_WR 8
#endif
// Row stride of the whole-body knot's H (the SRB knot's 6 x 6 H stays dense): 17 puts the
// rows R45 stores and the column R2 reads on distinct banks (tools/lds_bank_model_r3.py)
#ifndef MHPC_BWS_HS14
#define MHPC_BWS_HS14 14
#endif
template <int NX> constexpr int HStride = NX == 14 ? MHPC_BWS_HS14 : NX;
constexpr int WR = MHPC_BWS_WR;  // column stride of W (MHPC_BWS_WT)
__device__ __forceinline__ constexpr int widx(int r, int col) {
  return MHPC_BWS_WT ? col * WR + r : r * WS + col;
}
__device__ __forceinline__ constexpr int g2idx(int r, int col) {
  return MHPC_BWS_WT ? col * 2 + r : r * WS + col;
}
template <int NX> constexpr int JtStride = MHPC_BWS_WT ? (NX == 14 ? 18 : 10) : NX + MHPC_BWS_JTPAD;
constexpr int JtOff = MHPC_BWS_WT ? 1 : 0;
// The NU = 4 control rows of Q ([Qux | Quu | Qu]) column-major in U (MHPC_BWS_UT=1, default):
// R45 / R5 read a column of them (Qux[.][j], Qu) as two ds_read_b128 instead of four strided
// reads.  uidx(c, k) = row NX + k, column c.
#ifndef MHPC_BWS_UT
#define MHPC_BWS_UT 1
#endif
// Row stride of Q for the WB knot and column stride of U: bank spreading of R3's stores and
// R45's reads (tools/lds_bank_model_r3.py models every access of the whole-body knot: 575 ->
// 543 LDS-array cycles at 31 / 10 against 22 / 4; measured at batch 4096, k_bws<64,2,2>
// SQ_LDS_BANK_CONFLICT -18 %, SQ_LDS_IDX_ACTIVE -4.3 %, profiles/r03_bank_strides.txt)
#ifndef MHPC_BWS_QS14
#define MHPC_BWS_QS14 31
#endif
#ifndef MHPC_BWS_US
#define MHPC_BWS_US 10
#endif
template <int NX> struct QShape {
  static constexpr int NR = NX + 4;
  static constexpr int QS = NX == 14 ? MHPC_BWS_QS14 : 13;  // row stride of Q; column QV holds Qv
  static constexpr int QV = QS - 1;
};

// Arithmetic type of the 4x4 control block of a knot (adjugate, determinant, Quu^-1, the
// gains tq = Qux' Quu^-1 and the products that update H / G / dV with them): the solve's
// type, or double in the fp32 build (MHPC_BWS_WIDE, default; whole-body knots only): the fp32
// sweep's gains then carry the rounding of the fp32 Q blocks only, not of an fp32 inversion
// (C5 fp32: worst cost error vs the fp64 oracle 5.4e-3 -> 4.0e-3, gains after one sweep 3x
// closer in the stance phases).
#ifndef MHPC_BWS_WIDE
#define MHPC_BWS_WIDE 1
#endif
#if defined(MHPC_FP32) && MHPC_BWS_WIDE
using wreal = double;
#else
using wreal = real;
#endif

struct BwsLds {
  alignas(16) real H[14 * MHPC_BWS_HS14];
  alignas(16) real G[14];  // value function of knot k+1, then of knot k (row stride NX)
  alignas(16) real W[MHPC_BWS_WT ? WS * WR : 7 * WS];  // rows NQ..NX-1 of [A B] (widx)
  alignas(16) real G2[2 * WS];                         // stance rows of [C D] (g2idx)
  real l[JR];          // (lx, lu)
  real ldiag[18];      // diagonal running-cost Hessian (lxx, luu)
  real lyy2[4], ly2[2];
  union {
    struct {
      alignas(16) real Jt[JR * (MHPC_BWS_WT ? 18 : 15)];  // [A B]' H (NR x NX, JtStride<NX>)
      real Q[QR * MHPC_BWS_QS14];  // Qxx (NX x NX), Qux (rows NX.., cols ..NX), Quu; column QV = Qv
      alignas(16) real U[MHPC_BWS_QS14 * MHPC_BWS_US];  // rows NX..NX+3 of Q column-major (MHPC_BWS_UT)
    };
    struct {
      real H2[196];      // impact-aware step: lifted H' and (Px' H2)
      real Px[196];
      real T[196];
    };
  };
  real Qv[18];         // (Qx, Qu)
  real xb[14], ub[4], yb[4], posk;  // nominal knot + its position reference
  alignas(16) real Kst[56];          // results of the last knot, stored one knot later
  alignas(16) wreal inv[16];         // Quu^-1 (unsymmetrised), broadcast through LDS
  alignas(16) real dust[4];
  real hx[14], Hs[9], G2v[14];
  alignas(16) real junk[64];  // write target of the spare lanes of a round (never read)
  acc dV;
  int fail;
#ifdef MHPC_BWS_TIMING
  unsigned long long cyc[12], tlast;
#endif
};

// Q entry (row NX + k, column c): in U (MHPC_BWS_UT) or in Q (row stride qs)
__device__ __forceinline__ real& qu(BwsLds& sh, int qs, int nx, int k, int c) {
  return MHPC_BWS_UT ? sh.U[c * MHPC_BWS_US + k] : sh.Q[(nx + k) * qs + c];
}

// Optional cycle accounting per Riccati round (build with -DMHPC_BWS_TIMING; read with
// mhpc_dbg_bws_cycles): slot i accumulates the cycles since the previous mark.
#ifdef MHPC_BWS_TIMING
#define BWS_TMARK(sh, lane, i)                          \
  do {                                                  \
    if ((lane) == 0) {                                  \
      const unsigned long long t_ = clock64();          \
      (sh).cyc[i] += t_ - (sh).tlast;                   \
      (sh).tlast = t_;                                  \
    }                                                   \
  } while (0)
__device__ unsigned long long g_bws_cyc[12];
#else
#define BWS_TMARK(sh, lane, i) do { } while (0)
#endif

// Eigen-style 4x4 inverse by cofactors (same formulas as the oracle).
__device__ __forceinline__ void inverse4(const real* m, real* inv) {
  real a[16];
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
  const real det = m[0] * a[0] + m[1] * a[4] + m[2] * a[8] + m[3] * a[12];
#pragma unroll
  for (int i = 0; i < 16; ++i) inv[i] = a[i] / det;
}

// Eigen::LDLT(Quu - 1e-9 I).isPositive() (SinglePhase.cpp:202-209) on the lower triangle:
// ldlt_inplace<Lower>::unblocked with diagonal pivoting (first largest |diagonal|), the
// symmetric transposition applied to the lower triangle only, sign bookkeeping from
// ZeroSign; true iff no strictly negative pivot.  Branch-free (the pivot swaps are
// selects) so the scheduler can interleave it with the independent inverse / value-
// function work of the same round; same arithmetic as the oracle.
__device__ __forceinline__ void sel_swap(bool c, real& a, real& b) {
  const real ta = a, tb = b;
  a = c ? tb : ta;
  b = c ? ta : tb;
}
__device__ __forceinline__ bool ldlt_is_positive4(real* A) {
  int sign = 0;  // 0 ZeroSign, 1 PositiveSemiDef, 2 NegativeSemiDef, 3 Indefinite
  bool stop = false;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    int big = k;
    real bv = fabs(A[k * 5]);
#pragma unroll
    for (int i = k + 1; i < 4; ++i) {
      const real v = fabs(A[i * 5]);
      const bool gt = v > bv;
      bv = gt ? v : bv;
      big = gt ? i : big;
    }
#pragma unroll
    for (int I = k + 1; I < 4; ++I) {
      const bool sw = big == I;
#pragma unroll
      for (int j = 0; j < k; ++j) sel_swap(sw, A[k * 4 + j], A[I * 4 + j]);
#pragma unroll
      for (int i = I + 1; i < 4; ++i) sel_swap(sw, A[i * 4 + k], A[i * 4 + I]);
      sel_swap(sw, A[k * 5], A[I * 5]);
#pragma unroll
      for (int i = k + 1; i < I; ++i) sel_swap(sw, A[i * 4 + k], A[I * 4 + i]);
    }
    if (k > 0) {
      real temp[3];
#pragma unroll
      for (int j = 0; j < k; ++j) temp[j] = A[j * 5] * A[k * 4 + j];
      real s = 0;
#pragma unroll
      for (int j = 0; j < k; ++j) s += A[k * 4 + j] * temp[j];
      A[k * 5] -= s;
#pragma unroll
      for (int i = k + 1; i < 4; ++i) {
        real t = 0;
#pragma unroll
        for (int j = 0; j < k; ++j) t += A[i * 4 + j] * temp[j];
        A[i * 4 + k] -= t;
      }
    }
    const real akk = A[k * 5];
    const bool valid = fabs(akk) > real(0.0);
    if (k == 0) stop = !valid;  // whole diagonal zero: ZeroSign, stop
#pragma unroll
    for (int i = k + 1; i < 4; ++i) {
      const real q = A[i * 4 + k] / akk;
      A[i * 4 + k] = valid ? q : A[i * 4 + k];
    }
    int ns = sign;
    if (sign == 1) ns = akk < real(0.0) ? 3 : 1;
    else if (sign == 2) ns = akk > real(0.0) ? 3 : 2;
    else if (sign == 0) ns = akk > real(0.0) ? 1 : (akk < real(0.0) ? 2 : 0);
    sign = stop ? 0 : ns;
  }
  return sign == 1 || sign == 0;
}

// The verdict used by default (MHPC_BWS_PSD=1): an unpivoted LDL^T of the same matrix.
// By Sylvester's law of inertia its pivots have the signs of the pivoted factorisation's
// whenever no pivot is exactly zero, so the verdict is the same; a zero pivot leaves its
// column, as in Eigen.  A quarter of the instructions of the pivoted test (no pivot search
// or swaps, three reciprocals): -16 % backward-sweep time.  tests/test_psd_verdict.py
// checks the agreement on PD, indefinite, rank-deficient and near-singular matrices;
// MHPC_BWS_PSD=0 selects the pivoted restatement above.
#ifndef MHPC_BWS_PSD
#define MHPC_BWS_PSD 1
#endif
// MHPC_BWS_PSD_RCP (A/B): the pivots' reciprocals by the hardware estimate and two Newton
// steps (<= 1 ulp) instead of IEEE divisions -- the verdict only reads signs.
#ifndef MHPC_BWS_PSD_RCP
#define MHPC_BWS_PSD_RCP 0
#endif
__device__ __forceinline__ real fast_recip(real a) {
#if MHPC_BWS_PSD_RCP
  real r = __builtin_amdgcn_rcp(a);
  real e = fma(-a, r, real(1.0));
  r = fma(r, e, r);
  e = fma(-a, r, real(1.0));
  return fma(r, e, r);
#else
  return real(1.0) / a;
#endif
}
__device__ __forceinline__ bool ldlt_nopiv_is_positive4(real* A) {
  bool neg = false;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const real akk = A[k * 5];
    neg = neg || akk < real(0.0);
    const bool valid = akk != real(0.0);
    const real r = fast_recip(valid ? akk : real(1.0));
#pragma unroll
    for (int i = k + 1; i < 4; ++i) {
      const real l = A[i * 4 + k] * r;
#pragma unroll
      for (int j = k + 1; j <= i; ++j) A[i * 4 + j] -= valid ? l * A[j * 4 + k] : real(0.0);
    }
  }
  return !neg;
}

// Value of lane `src` (uniform) of a value held per lane: readlanes, no LDS.
__device__ __forceinline__ float lane_bcast(float v, int src) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), src));
}
__device__ __forceinline__ double lane_bcast(double v, int src) {
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, src);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), src);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Row coefficient of the exact part of [A B] (see file header).
template <int NQ>
__device__ __forceinline__ real coef_a(int col, real dt) {
  return col < NQ ? real(1.0) : (col < 2 * NQ ? dt : real(0.0));
}
template <int NQ>
__device__ __forceinline__ int coef_b(int col) {
  return col < NQ ? col : col - NQ;
}

// One Riccati knot.  On entry sh.{W,G2,l,lxx,luu,lyy2,ly2} hold the knot's derivatives and
// sh.{H,G} the value function of knot k+1; on exit sh.{H,G} hold that of knot k.
#ifndef MHPC_BWS_CH2
#define MHPC_BWS_CH2 5
#endif
#ifndef MHPC_BWS_CH3
#define MHPC_BWS_CH3 2
#endif
#ifndef MHPC_BWS_CH5
#define MHPC_BWS_CH5 4
#endif
constexpr int CH2 = MHPC_BWS_CH2, CH3 = MHPC_BWS_CH3, CH5 = MHPC_BWS_CH5;
#ifndef MHPC_BWS_INVLDS
#define MHPC_BWS_INVLDS 1
#endif

// r2x / r45x: the caller's per-knot side work, run inside the R2 and R45 rounds (before
// their barriers) so it needs no round of its own -- global traffic of the knot pipeline
// (stores of the previous knot, prefetch of the next) and the drop of the next knot's
// derivatives into LDS (nothing of R45 reads those arrays).
template <int NT, int NQ, bool HAS_Y, class R2X, class R45X>
__device__ bool riccati_knot(BwsLds& sh, int lane, real dt, real reg, real eps9, R2X&& r2x,
                             R45X&& r45x) {
  constexpr int NX = 2 * NQ, NR = NX + 4;
  constexpr int QS = QShape<NX>::QS, QV = QShape<NX>::QV;
  // the control block's arithmetic type: wreal for the whole-body knots (the fp32 sweep's
  // gain errors come from them: tools/diag_fp32_stages.py), the solve's type for SRB knots
  using wk = typename std::conditional<NQ == 7, wreal, real>::type;
  // R2: Jt = [A B]' H (NR x NX) and Qv = (l + [A B]' G) + [C D]' ly, G taken as column NX
  // of [H | G].  Lane = (column j, row group g): the column stays in registers and the lane
  // runs T2 independent row chains.
  {
    constexpr int NC = NX + 1, GR = NT / NC, T2 = (NR + GR - 1) / GR;
    static_assert(GR * T2 <= JR && GR * T2 <= QR && GR * T2 <= WS, "R2 padding");
    const int j = lane % NC, g = lane / NC;
    const bool isg = j == NX;
    const bool wr = g < GR;                    // spare lanes write to the junk row
    const real* col0 = isg ? sh.G : sh.H + j;  // [H | G] column j, element b at col0[b*cs]
    real hc[NQ];
#pragma unroll
    for (int r = 0; r < NQ; ++r) hc[r] = col0[isg ? NQ + r : (NQ + r) * HStride<NX>];
    real ly0 = real(0.0), ly1 = real(0.0);
    if (HAS_Y) { ly0 = sh.ly2[0]; ly1 = sh.ly2[1]; }
    // straight-line rows (no per-row branches, so the scheduler interleaves the T2 chains):
    // the G-column extras are computed on every lane and selected
    constexpr int C = T2 < CH2 ? T2 : CH2;
#pragma unroll
    for (int t0 = 0; t0 < T2; t0 += C) {
      real acc[C];
#pragma unroll
      for (int u = 0; u < C; ++u) {
        if (t0 + u >= T2) continue;
        const int row = g + GR * (t0 + u);  // < JR
        const real a = coef_a<NQ>(row, dt);
        const int bi = coef_b<NQ>(row);
        const real hb = col0[isg ? bi : bi * HStride<NX>];
        real sacc = a != real(0.0) ? a * hb : real(0.0);
#pragma unroll
        for (int r = 0; r < NQ; ++r) sacc += sh.W[widx(r, row)] * hc[r];
        real tt = real(0.0);
        if (HAS_Y) tt = sh.G2[g2idx(0, row)] * ly0 + sh.G2[g2idx(1, row)] * ly1;
        const real gs = (sh.l[row] + sacc) + tt;
        acc[u] = isg ? gs : sacc;
      }
#pragma unroll
      for (int u = 0; u < C; ++u) {
        if (t0 + u >= T2) continue;
        const int row = g + GR * (t0 + u);
        real* dqv = &sh.Q[row * QS + QV];
        if (MHPC_BWS_UT)  // Qu rows to U; padding rows (>= NR) to the junk slot
          dqv = row < NX ? dqv : row < NR ? &sh.U[QV * MHPC_BWS_US + (row - NX)] : &sh.junk[lane & 63];
        real* dst = isg ? dqv : &sh.Jt[row * JtStride<NX> + JtOff + j];
        *(wr ? dst : &sh.junk[lane & 63]) = acc[u];
      }
    }
  }
  BWS_TMARK(sh, lane, NQ == 3 ? 4 : 3);
  r2x();
  __syncthreads();
  BWS_TMARK(sh, lane, NQ == 3 ? 8 : 1);
  // R3: Qxx = (lxx + C'lyy C) + A'HA ; Qux = (0 + D'lyy C) + B'HA ; Quu = (luu + D'lyy D) + B'HB
  // (+ reg on the diagonal).  Lane = (row of Jt, column group g), the row Jt[row, NQ..] in
  // registers, T3 independent column chains.
  {
    constexpr int RG = NT / NR, T3 = (NR + RG - 1) / RG;  // columns g + RG t < QV
    static_assert(RG * T3 <= QV && RG * T3 <= WS, "R3 padding");
    const int row = lane % NR, g = lane / NR;
    const bool wr = g < RG;
    real jr[NQ];
#pragma unroll
    for (int r = 0; r < NQ; ++r) jr[r] = sh.Jt[row * JtStride<NX> + JtOff + NQ + r];
    real c0 = real(0.0), c1 = real(0.0);
    if (HAS_Y) {
      const real gr0 = sh.G2[g2idx(0, row)], gr1 = sh.G2[g2idx(1, row)];
      c0 = gr0 * sh.lyy2[0] + gr1 * sh.lyy2[2];
      c1 = gr0 * sh.lyy2[1] + gr1 * sh.lyy2[3];
    }
    const real dg = sh.ldiag[row];
    constexpr int C = T3 < CH3 ? T3 : CH3;
#pragma unroll
    for (int t0 = 0; t0 < T3; t0 += C) {
      real acc[C];
#pragma unroll
      for (int u = 0; u < C; ++u) {
        if (t0 + u >= T3) continue;
        const int col = g + RG * (t0 + u);
        const real a = coef_a<NQ>(col, dt);
        const real jb = sh.Jt[row * JtStride<NX> + JtOff + coef_b<NQ>(col)];
        real sacc = a != real(0.0) ? a * jb : real(0.0);
#pragma unroll
        for (int r = 0; r < NQ; ++r) sacc += jr[r] * sh.W[widx(r, col)];
        const real base = row == col ? dg : real(0.0);
        real e2 = real(0.0);
        if (HAS_Y) e2 = c0 * sh.G2[g2idx(0, col)] + c1 * sh.G2[g2idx(1, col)];
        real v = (base + e2) + sacc;
        const real vr = v + real(1.0) * reg;
        acc[u] = row == col ? vr : v;
      }
#pragma unroll
      for (int u = 0; u < C; ++u) {
        if (t0 + u >= T3) continue;
        const int col = g + RG * (t0 + u);
        real* dq = MHPC_BWS_UT && row >= NX ? &sh.U[col * MHPC_BWS_US + (row - NX)] : &sh.Q[row * QS + col];
        *(wr ? dq : &sh.junk[lane & 63]) = acc[u];
      }
    }
  }
  __syncthreads();
  BWS_TMARK(sh, lane, NQ == 3 ? 9 : 2);
  // R45: PSD test of Quu - 1e-9 I (every lane, registers, static indices); adjugate of Quu
  // spread over lanes 0..15 (one 3x3 minor each) and broadcast back with readlane (no LDS
  // round trip); then, in the same round, tq = Qux' Quu_inv, K = -tq', du, dV and
  // H = sym(Qxx) - tq Qux, G = Qx - tq Qu.
  wk q0[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) q0[c] = qu(sh, QS, NX, 0, NX + c);
  wk adj = wk(0.0);
  bool psd;
  {
    // the PSD verdict is applied at the end of the round: a failed knot abandons the sweep
    // (everything written here is rewritten by the retry), only dV must stay untouched
    const int i = (lane >> 2) & 3, j = lane & 3;  // lanes 0..15 of every wave
    const int r0 = j == 0 ? 1 : 0, r1 = j <= 1 ? 2 : 1, r2 = j <= 2 ? 3 : 2;
    const int c0 = i == 0 ? 1 : 0, c1 = i <= 1 ? 2 : 1, c2 = i <= 2 ? 3 : 2;
#define QM(r, c) qu(sh, QS, NX, r, NX + (c))
    const wk m00 = QM(r0, c0), m01 = QM(r0, c1), m02 = QM(r0, c2);
    const wk m10 = QM(r1, c0), m11 = QM(r1, c1), m12 = QM(r1, c2);
    const wk m20 = QM(r2, c0), m21 = QM(r2, c1), m22 = QM(r2, c2);
#undef QM
    real A[16];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        A[a * 4 + c] = qu(sh, QS, NX, a, NX + c) - (a == c ? real(1.0) * eps9 : real(0.0));
#if MHPC_BWS_PSD == 1
    psd = ldlt_nopiv_is_positive4(A);
#elif MHPC_BWS_PSD == 2
    psd = A[0] > -real(1e300);  // timing experiment only: no PSD test
#else
    psd = ldlt_is_positive4(A);
#endif
    // adj[i][j] = (-1)^(i+j) det(minor without row j, column i)
    const wk det3 = m00 * (m11 * m22 - m12 * m21) - m01 * (m10 * m22 - m12 * m20) +
                         m02 * (m10 * m21 - m11 * m20);
    adj = ((i + j) & 1) ? -det3 : det3;
  }
  const wk det = q0[0] * lane_bcast(adj, 0) + q0[1] * lane_bcast(adj, 4) +
                      q0[2] * lane_bcast(adj, 8) + q0[3] * lane_bcast(adj, 12);
  const wk invl = adj / det;
  wk Qi[16];
  {
    wk inv[16];  // unsymmetrised inverse (uniform)
#if MHPC_BWS_INVLDS
    // through LDS: 16 readlane pairs would hold the inverse in 32 SGPRs, which the kernel's
    // SGPR file cannot spare (it spills to VGPR lanes elsewhere in the knot loop)
    // Lanes 0..15 store, every lane reads all 16 back, within one wave (NT == 64): the
    // wave's LDS operations complete in issue order, and the compiler keeps the loads
    // behind the store because they may alias it (same array, lane-dependent index).  Any
    // explicit ordering costs: a wave barrier (a scheduling barrier) +9 % backward-sweep
    // time, wavefront-scope fences +9 %, volatile accesses +28 % (MHPC_BWS_WAVEBAR = 1 / 3
    // builds; A/B at batch 1024 in profiles/r02_ab_inverse_broadcast.txt).
#ifndef MHPC_BWS_WAVEBAR
#define MHPC_BWS_WAVEBAR 0
#endif
    // spare lanes: the junk slot (a two-slot one when wk is wider than real)
    wreal* const jk = reinterpret_cast<wreal*>(
        &sh.junk[std::is_same<wreal, real>::value ? (lane & 63) : (lane & 62)]);
    *(lane < 16 ? &sh.inv[lane] : jk) = wreal(invl);
    if (NT > 64) __syncthreads();
#if MHPC_BWS_WAVEBAR == 1
    else __builtin_amdgcn_wave_barrier();
#elif MHPC_BWS_WAVEBAR == 3
    else {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
#endif
#pragma unroll
    for (int e = 0; e < 16; ++e) inv[e] = sh.inv[e];
#else
#pragma unroll
    for (int e = 0; e < 16; ++e) inv[e] = lane_bcast(invl, e);
#endif
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) Qi[a * 4 + c] = (inv[a * 4 + c] + inv[c * 4 + a]) / 2;
    // dV += -Qu' inv Qu, unsymmetrised inverse, no 1/2 (MHPC_CompoundTypes.h:142)
    wk s = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      wk t = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) t += qu(sh, QS, NX, k, QV) * inv[k * 4 + c];
      s += t * qu(sh, QS, NX, c, QV);
    }
    // s and psd are uniform: every lane of wave 0 writes the same value (no divergent
    // branch); the other waves of a 128-thread block must not re-read the updated dV
    const acc dv0 = sh.dV;
    acc* const jd = reinterpret_cast<acc*>(
        &sh.junk[std::is_same<acc, real>::value ? (lane & 63) : (lane & 62)]);
    *(lane < 64 ? &sh.dV : jd) = psd ? acc(dv0 + -s) : dv0;
  }
  {
    // lane = (row i of [Qux | Qu]' , column group g); row NX stands for Qu (du), column NX
    // of the update for G.  tq row i in registers; K[c][i] = -tq[i][c] exactly (Qi is
    // symmetric and the sums run in the same order).
    constexpr int NI = NX + 1, GC = NT / NI, T5 = (NX + 1 + GC - 1) / GC;
    const int i = lane % NI, g = lane / NI;
    const int si = i < NX ? i : QV;
    wk qi[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) qi[k] = qu(sh, QS, NX, k, si);
    wk tq[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      wk t = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) t += qi[k] * Qi[k * 4 + c];
      tq[c] = t;
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
      *(g == 0 ? (i < NX ? &sh.Kst[c * NX + i] : &sh.dust[c]) : &sh.junk[lane & 63]) = real(-tq[c]);
    constexpr int C = T5 < CH5 ? T5 : CH5;
#pragma unroll
    for (int t0 = 0; t0 < T5; t0 += C) {
      real acc[C];
#pragma unroll
      for (int u = 0; u < C; ++u) {
        if (t0 + u >= T5) continue;
        const int j = g + GC * (t0 + u);
        const int sj = j < NX ? j : QV;
        wk sacc = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) sacc += tq[c] * qu(sh, QS, NX, c, sj);
        const real qij = sh.Q[i * QS + sj];
        const real qji = sh.Q[(j < NX ? j : 0) * QS + i];
        const real sym = (qij + qji) / 2;
        const real base = j < NX ? sym : qij;
        acc[u] = real(base - sacc);
      }
#pragma unroll
      for (int u = 0; u < C; ++u) {
        if (t0 + u >= T5) continue;
        const int j = g + GC * (t0 + u);
        const bool wr = g < GC && i < NX && j <= NX;
        *(wr ? (j < NX ? &sh.H[i * HStride<NX> + j] : &sh.G[i]) : &sh.junk[lane & 63]) = acc[u];
      }
    }
  }
  BWS_TMARK(sh, lane, NQ == 3 ? 6 : 5);
  r45x();
  __syncthreads();
  BWS_TMARK(sh, lane, NQ == 3 ? 10 : 7);
  return psd;
}

// Running-cost derivatives of a WB knot: lx / lxx per state lane (CostBase.cpp:28-31),
// the control / force part comes precomputed with the partials record (see mhpc_solver.h).
// The lane's weight and fixed reference are loaded once per phase (wb_cost_x_consts): a
// lane-indexed __constant__ read inside the knot loop is a vector memory load whose wait
// would also drain the knot's prefetch and stores.
struct CostXConsts {
  real w2;   // 2 dt Q[i]
  real rx;   // reference of state i (unused for i = 0: the position reference)
};
__device__ __forceinline__ CostXConsts wb_cost_x_consts(int lane, const SolveParams& sp, int mode,
                                                        real dt) {
  CostXConsts c{real(0.0), real(0.0)};
  if (lane < 14) {
    const int i = lane;
    c.rx = i == 1 ? sp.height : i == 2 ? real(0.0) : (i >= 3 && i < 7) ? cQjointBias[i - 3]
           : i == 7 ? sp.vel : real(0.0);
    c.w2 = 2 * dt * sp.cw.wQ[mode - 1][i];
  }
  return c;
}
__device__ __forceinline__ void wb_cost_x(BwsLds& sh, int lane, const CostXConsts& c, real pos) {
  if (lane < 14) {
    const real rxi = lane == 0 ? pos : c.rx;
    sh.l[lane] = c.w2 * (sh.xb[lane] - rxi);
    sh.ldiag[lane] = c.w2;
  }
}

// SRB Jacobian entry of row 3+r, column col of [A B] (FBDynamics_par.c operation order).
__device__ __forceinline__ real srb_w_entry(int r, int col, const real* x, const real* u,
                                              const real* p, const real* s, real dt) {
  MHPC_NO_FMA
  const int row = 3 + r;
  real ac = real(0.0);
  if (col < 6) {
    if (row == 5 && col == 0) ac = s[0] * (kSrbInvInertia * u[1]) + s[1] * (kSrbInvInertia * u[3]);
    if (row == 5 && col == 1) ac = -(s[0] * (kSrbInvInertia * u[0]) + s[1] * (kSrbInvInertia * u[2]));
    return (col == row ? real(1.0) : real(0.0)) + ac * dt;
  }
  const int c = col - 6;
  real bc = real(0.0);
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

// Terminal value function of phase p (SinglePhase.cpp:189-191): G = Phix + Gnext,
// H = Phixx + Hnext, with Gnext/Hnext in sh.G/sh.H; AL partials only while st->al_partials
// (quirk B1: forward_sweep_partials_only does not add them).
template <int NT, int NX>
__device__ void terminal_value(const SolveParams& sp, const ProbState* st, BwsLds& sh, int lane,
                               int p, real pos, const real* xe, real* Gout) {
  constexpr bool wb = NX == 14;
  const int mode = sp.mode[p];
  const bool al = wb && ntc_of(mode, true) && sp.AL_active && st->al_partials;
  real h = 0;
  if (al && lane == 0) {
    real hx[14], Hs[3][3];
    if (mode == 2) wb_touchdown_compact<kFront>(xe, &h, hx, Hs);
    else wb_touchdown_compact<kBack>(xe, &h, hx, Hs);
#pragma unroll
    for (int i = 0; i < 14; ++i) sh.hx[i] = hx[i];
#pragma unroll
    for (int i = 0; i < 9; ++i) sh.Hs[i] = Hs[i / 3][i % 3];
    sh.G2v[0] = h;
  }
  __syncthreads();
  if (al) h = sh.G2v[0];
  const real s = st->sigma[p], lam = st->lambda[p];
  const int ih = mode == 2 ? 3 : 5;  // touchdown Hessian block (theta, hip, knee)
  #pragma unroll 1
  for (int e = lane; e < NX * NX + NX; e += NT) {
    if (e < NX * NX) {
      const int i = e / NX, j = e - i * NX;
      real v = i == j ? (wb ? sp.cw.wQf[mode - 1][i] : sp.cw.fQf[mode - 1][i]) : real(0.0);
      if (al) {
        const int ai = i == 2 ? 0 : (i == ih ? 1 : (i == ih + 1 ? 2 : -1));
        const int aj = j == 2 ? 0 : (j == ih ? 1 : (j == ih + 1 ? 2 : -1));
        const real hij = (ai >= 0 && aj >= 0) ? sh.Hs[ai * 3 + aj] : real(0.0);
        v += 50 * (s * s / 2 * (sh.hx[i] * sh.hx[j] + h * hij) + lam * hij);
      }
      sh.H[i * HStride<NX> + j] = v + sh.H[i * HStride<NX> + j];
    } else {
      const int i = e - NX * NX;
      real rxi;
      if (wb) rxi = i == 0 ? pos : (i == 7 ? sp.vel : cXtermWB[mode - 1][i]);
      else rxi = i == 0 ? pos : (i == 1 ? sp.height : (i == 3 ? sp.vel : real(0.0)));
      real v = (wb ? sp.cw.wQf[mode - 1][i] : sp.cw.fQf[mode - 1][i]) * (xe[i] - rxi);
      if (al) v += 50 * (s * s / 2 * sh.hx[i] * h + lam * sh.hx[i]);
      const real g = v + sh.G[i];
      sh.G[i] = g;
      Gout[i] = g;
    }
  }
  __syncthreads();
}

// impact_aware_step (MultiPhaseDDP.cpp:300-341) for a WB phase p: sh.G/H hold CTG[0] of
// phase p+1 (6-dim if that phase is SRB); on exit the 14-dim Gnext/Hnext of phase p.
template <int NT>
__device__ void impact_step(const SolveParams& sp, const DevBufs& d, int b, BwsLds& sh, int lane,
                            int p, int64_t* px_reads) {
  const int mode = sp.mode[p];
  const bool nwb = p + 1 < sp.n_wb;
  const bool imp = mode == 2 || mode == 4;
  // lift to the full-model space: E' G', E' H' E (E = _stateProj for an SRB next phase)
  #pragma unroll 1
  for (int e = lane; e < 196 + 14; e += NT) {
    if (e < 196) {
      const int i = e / 14, j = e - i * 14;
      real v;
      if (nwb) v = sh.H[i * HStride<14> + j];
      else {
        const int pi = i < 3 ? i : (i >= 7 && i < 10 ? i - 4 : -1);
        const int pj = j < 3 ? j : (j >= 7 && j < 10 ? j - 4 : -1);
        v = (pi >= 0 && pj >= 0) ? sh.H[pi * 6 + pj] : real(0.0);
      }
      sh.H2[e] = v;
    } else {
      const int i = e - 196;
      real v;
      if (nwb) v = sh.G[i];
      else {
        const int q = i < 3 ? i : (i >= 7 && i < 10 ? i - 4 : -1);
        v = q >= 0 ? sh.G[q] : real(0.0);
      }
      sh.G2v[i] = v;
    }
  }
  if (imp) {
    const real* pxc = d.px + ((size_t)b * MAXP + p) * 196;  // column-major
    #pragma unroll 1
    for (int e = lane; e < 196; e += NT) sh.Px[(e % 14) * 14 + e / 14] = pxc[e];
    if (lane == 0) ++*px_reads;
  }
  __syncthreads();
  if (imp) {
    // G = Px' G2 ; T = Px' H2 ; H = T Px
    #pragma unroll 1
    for (int e = lane; e < 196 + 14; e += NT) {
      if (e < 196) {
        const int i = e / 14, j = e - i * 14;
        real s = 0;
#pragma unroll
        for (int m = 0; m < 14; ++m) s += sh.Px[m * 14 + i] * sh.H2[m * 14 + j];
        sh.T[e] = s;
      } else {
        const int i = e - 196;
        real s = 0;
#pragma unroll
        for (int m = 0; m < 14; ++m) s += sh.Px[m * 14 + i] * sh.G2v[m];
        sh.G[i] = s;
      }
    }
    __syncthreads();
    #pragma unroll 1
    for (int e = lane; e < 196; e += NT) {
      const int i = e / 14, j = e - i * 14;
      real s = 0;
#pragma unroll
      for (int m = 0; m < 14; ++m) s += sh.T[i * 14 + m] * sh.Px[m * 14 + j];
      sh.H[i * HStride<14> + j] = s;
    }
  } else {
    #pragma unroll 1
    for (int e = lane; e < 196; e += NT) sh.H[(e / 14) * HStride<14> + e % 14] = sh.H2[e];
    if (lane < 14) sh.G[lane] = sh.G2v[lane];
  }
  __syncthreads();
}

// s_waitcnt vmcnt(0) with expcnt / lgkmcnt left at their maxima (gfx9 encoding)
constexpr int kVmcnt0 = 0x0F70;

#ifdef MHPC_FP32
using real2 = float2;
#else
using real2 = double2;
#endif
// Store the staged K / du / G of knot record `rec`.  All global traffic of a knot (these
// stores and the prefetch loads of the next record) is issued back to back right after the
// wait for the previous prefetch, so the next wait (a full knot later) finds both retired:
// gfx950 keeps one in-order VM counter for loads and stores.
// Per-lane part of flush_knot, fixed for a phase: one 2-wide store per lane, one store
// instruction per knot: K (2 NX pairs), du (2), G (NX / 2).  Lanes past them repeat lane 0's
// store (same address, same value), so the store needs no divergent branch.
struct FlushLane {
  real* base;   // d.K / d.du / d.G
  int stride;   // reals per knot record of that array
  int o;        // pair offset (reals) inside the record
  int src;      // staged source in the LDS block (reals from its start)
};
template <int NX>
__device__ __forceinline__ FlushLane flush_lane(const DevBufs& d, const BwsLds& sh, int lane) {
  constexpr int NK2 = 2 * NX, NG2 = NX / 2;
  const int l = lane < NK2 + 2 + NG2 ? lane : 0;
  const bool isk = l < NK2, isd = !isk && l < NK2 + 2;
  FlushLane f;
  f.o = 2 * (isk ? l : isd ? l - NK2 : l - NK2 - 2);
  f.base = isk ? d.K : isd ? d.du : d.G;
  f.stride = isk ? 56 : isd ? 4 : 14;
  const real* src = isk ? sh.Kst : isd ? sh.dust : sh.G;
  f.src = (int)(src - reinterpret_cast<const real*>(&sh)) + f.o;
  return f;
}
template <int NT, int NX>
__device__ __forceinline__ void flush_knot(size_t rec, const BwsLds& sh, const FlushLane& f) {
#ifdef MHPC_BWS_NOSTORE
  return;  // timing experiment only
#endif
  static_assert(2 * NX + 2 + NX / 2 <= NT, "flush lanes");
  *reinterpret_cast<real2*>(f.base + rec * f.stride + f.o) =
      *reinterpret_cast<const real2*>(reinterpret_cast<const real*>(&sh) + f.src);
}

// Backward sweep of one WB phase: knots N-2..0 with a one-knot register prefetch.
// STANCE: a stance phase (modes 1, 3) carries the contact-force outputs y (C, D, ly, lyy);
// one loop per variant keeps each variant's hoisted lane addresses out of the other's.
template <int NT, bool STANCE>
__device__ bool sweep_wb_phase(const SolveParams& sp, const DevBufs& d, int b, const ProbState* st,
                               BwsLds& sh, int lane, int p, real reg, int64_t* knots) {
  const int N = sp.N[p], ko = sp.ko[p];
  const real dt = sp.dt[p];
  const int nom = st->nom_slot;
  constexpr bool stance = STANCE;
  const real* pos = d.refpos + (size_t)b * sp.NK + ko;
  // prefetch registers: PT doubles of the partials record + 1 of the nominal knot
  constexpr int PT = (PS + NT - 1) / NT;
  real pre[PT], prex = 0;
  real* const shf = reinterpret_cast<real*>(&sh);
  const int junk = (int)(sh.junk - shf) + (lane & 63);
  const int xo = lane < 22 ? lane : 0;
  const bool isref = lane == 22;
  auto load = [&](int k) {
    const real* prec = d.par + ((size_t)b * sp.NK + ko + k) * PS;
#pragma unroll
    for (int t = 0; t < PT; ++t) {
      const int e = lane + NT * t;
      pre[t] = prec[e < PS ? e : PS - 1];  // unconditional: no exec-masked load
    }
    const real* tk = traj_ptr(sp, d, b, nom, ko + k);
    prex = *(isref ? pos + k : tk + xo);
  };
  const CostXConsts cx = wb_cost_x_consts(lane, sp, sp.mode[p], dt);
  // Where each prefetched record element goes, fixed for the phase: value = pre * mul + base
  // into the LDS block at dst (W entries: (I + dt Ac | dt Bc), everything else verbatim:
  // x * 1 + (-0) == x exactly); elements with no target write the lane's junk slot.
  int dst[PT];
  real mul[PT], base[PT];
#pragma unroll
  for (int t = 0; t < PT; ++t) {
    const int e = lane + NT * t;
    dst[t] = junk;
    mul[t] = real(1.0);
    base[t] = -real(0.0);
    if (e < PS_JAC) {
      const int col = e / 9, r = e - col * 9;
      if (r < 7) {
        dst[t] = (int)(sh.W - shf) + widx(r, col);
        mul[t] = dt;
        base[t] = col == 7 + r ? real(1.0) : real(0.0);
      } else if (stance) {
        dst[t] = (int)(sh.G2 - shf) + g2idx(r - 7, col);
      }
    } else if (e < PS) {
      const int q = e - PS_JAC;  // lu 4, luu 4, ly 2, lyy 4
      dst[t] = q < 4 ? (int)(sh.l - shf) + 14 + q
             : q < 8 ? (int)(sh.ldiag - shf) + 14 + q - 4
             : q < 10 ? (int)(sh.ly2 - shf) + q - 8 : (int)(sh.lyy2 - shf) + q - 10;
    }
  }
  // lxx = 2 dt Q is constant over the phase (CostBase.cpp:28-31)
  if (lane < 14) sh.ldiag[lane] = cx.w2;
  const int dlx = lane < 14 ? (int)(sh.l - shf) + lane : junk;
  // drop the prefetched knot into LDS: W = rows 7..13 of [I + dt Ac | dt Bc], G2 = [C D],
  // the control / force cost derivatives, and lx from the nominal state in prex
  // (CostBase.cpp:28-31; lane 22 holds the position reference)
  auto drop = [&]() {
    __builtin_amdgcn_s_waitcnt(kVmcnt0);  // the prefetch (and the stores issued before it)
#pragma unroll
    for (int t = 0; t < PT; ++t) shf[dst[t]] = __builtin_fma(pre[t], mul[t], base[t]);
    const real pk = lane_bcast(prex, 22);
    const real rxi = lane == 0 ? pk : cx.rx;
    shf[dlx] = cx.w2 * (prex - rxi);
  };
  const FlushLane fl = flush_lane<14>(d, sh, lane);
  load(N - 2);
  drop();
  __syncthreads();
  for (int k = N - 2; k >= 0; --k) {
    const int kk = ko + k;
    auto r2x = [&]() {
      if (k < N - 2) flush_knot<NT, 14>((size_t)b * sp.NK + kk + 1, sh, fl);
      if (k > 0) load(k - 1);
    };
    auto r45x = [&]() {
      if (k > 0) drop();
    };
    const bool ok = riccati_knot<NT, 7, STANCE>(sh, lane, dt, reg, sp.eps9, r2x, r45x);
    ++*knots;
    if (!ok) return false;
  }
  if (N >= 2) flush_knot<NT, 14>((size_t)b * sp.NK + ko, sh, fl);
  return true;
}

template <int NT>
__device__ bool sweep_fb_phase(const SolveParams& sp, const DevBufs& d, int b, const ProbState* st,
                               BwsLds& sh, int lane, int p, real reg, int64_t* knots) {
  const int N = sp.N[p], ko = sp.ko[p], mode = sp.mode[p];
  const real dt = sp.dt[p];
  const int nom = st->nom_slot;
  const real* pos = d.refpos + (size_t)b * sp.NK + ko;
  real foot[4], cs[2];
  plan_foothold(traj_ptr(sp, d, b, nom, ko), dt * N, mode, foot);
  srb_contact(mode, cs);
  const int m = mode - 1;
  // per-lane cost weight 2 dt Q (lanes 30..35: state i) / 2 dt R (lanes 36..39: control c)
  // and fixed reference, hoisted out of the knot loop (see wb_cost_x_consts)
  real fb_w2 = real(0.0), fb_rx = real(0.0);
  if (lane >= 30 && lane < 36) {
    const int i = lane - 30;
    fb_w2 = 2 * dt * sp.cw.fQ[m][i];
    fb_rx = i == 1 ? sp.height : i == 3 ? sp.vel : real(0.0);
  } else if (lane >= 36 && lane < 40) {
    const int c = lane - 36;
    fb_w2 = 2 * dt * sp.cw.fR[m][c];
    fb_rx = (c == 1 || c == 3) ? real(8.252) * real(9.81) : real(0.0);
  }
  // every wave of the block loads the same nominal words (lane & 63), so the uniform W
  // entries of the drop below are the same values whichever wave writes them
  const int xo = (lane & 63) < 10 ? (lane & 63) : 0;
  const bool isref = (lane & 63) == 10;
  auto loadx = [&](int k) {  // unconditional single load per lane (no exec-masked load)
    const real* tk = traj_ptr(sp, d, b, nom, ko + k);
    return *(isref ? pos + k : tk + xo);
  };
  real* const shf = reinterpret_cast<real*>(&sh);
  const int junk = (int)(sh.junk - shf) + (lane & 63);
  // cost derivative slot of the lane (lanes 30..35: lx of state i, 36..39: lu of control c)
  const int dl = lane >= 30 && lane < 40 ? (int)(sh.l - shf) + lane - 30 : junk;
  const int shsrc = lane >= 30 && lane < 40 ? lane - 30 : 0;
  // lxx / luu = 2 dt Q / 2 dt R are constant over the phase
  if (lane >= 30 && lane < 40) sh.ldiag[lane - 30] = fb_w2;
  // drop of knot k: the nominal (x 6, u 4) and position reference sit in prex of lanes
  // 0..10; W rows (FBDynamics_par.c order) and the cost derivatives straight from registers.
  // Only six entries of W (row 5: the torque terms) depend on the knot: they are uniform,
  // so every lane computes and writes them; the rest is written once per phase (full).
  auto drop = [&](real px, bool full) {
    __builtin_amdgcn_s_waitcnt(kVmcnt0);
    const real xs[2] = {lane_bcast(px, 0), lane_bcast(px, 1)};
    const real us[4] = {lane_bcast(px, 6), lane_bcast(px, 7), lane_bcast(px, 8),
                          lane_bcast(px, 9)};
    const real pk = lane_bcast(px, 10);
    const real own = __shfl(px, shsrc);
    if (full) {
      if (lane < 30) {
        const int r = lane / 10, col = lane - r * 10;
        sh.W[widx(r, col)] = srb_w_entry(r, col, xs, us, foot, cs, dt);
      }
    } else {
      sh.W[widx(2, 0)] = srb_w_entry(2, 0, xs, us, foot, cs, dt);
      sh.W[widx(2, 1)] = srb_w_entry(2, 1, xs, us, foot, cs, dt);
#pragma unroll
      for (int c = 6; c < 10; ++c) sh.W[widx(2, c)] = srb_w_entry(2, c, xs, us, foot, cs, dt);
    }
    const real rxi = lane == 30 ? pk : fb_rx;
    shf[dl] = fb_w2 * (own - rxi);
  };
  const FlushLane fl = flush_lane<6>(d, sh, lane);
  real prex = loadx(N - 2);
  drop(prex, true);
  __syncthreads();
  for (int k = N - 2; k >= 0; --k) {
    const int kk = ko + k;
    auto r2x = [&]() {
      if (k < N - 2) flush_knot<NT, 6>((size_t)b * sp.NK + kk + 1, sh, fl);
      if (k > 0) prex = loadx(k - 1);
    };
    auto r45x = [&]() {
      if (k > 0) drop(prex, false);
    };
    const bool ok = riccati_knot<NT, 3, false>(sh, lane, dt, reg, sp.eps9, r2x, r45x);
    ++*knots;
    if (!ok) return false;
  }
  if (N >= 2) flush_knot<NT, 6>((size_t)b * sp.NK + ko, sh, fl);
  return true;
}

// One sweep attempt with regularisation reg.  PART 0: every phase, from a zero terminal
// value function (MultiPhaseDDP::backward_sweep).  PART 1: only the SRB phases (P-1 ..
// n_wb), which read no partials record, so this launch can run beside the partials of the
// same iteration.  PART 2: the WB phases (n_wb-1 .. 0), resuming from the value function
// PART 1 left in d.carry.  PART 1 then PART 2 is PART 0's arithmetic, bit for bit (the
// carried H / G / dV are stored and reloaded exactly).
template <int NT, int PART>
__device__ bool bws_sweep(const SolveParams& sp, const DevBufs& d, int b, ProbState* st, BwsLds& sh,
                          real reg, int64_t* knots, int64_t* knots_wb, int64_t* px_reads,
                          bool from_carry = true) {
  const int lane = threadIdx.x;
  const int nom = st->nom_slot;
  if (PART == 2) {
    // resume: the value function from d.carry, or as a PART 1 sweep of this kernel left it
    const BwsCarry& c = d.carry[b];
    if (from_carry) {
      #pragma unroll 1
      for (int e = lane; e < 196; e += NT) sh.H[e] = c.H[e];
      if (lane < 14) sh.G[lane] = c.G[lane];
    }
  } else {
    #pragma unroll 1
    for (int e = lane; e < 14 * MHPC_BWS_HS14; e += NT) sh.H[e] = 0;  // Gnext = 0, Hnext = 0 (last phase)
    if (lane < 14) sh.G[lane] = 0;
    if (lane == 0) sh.dV = 0;
  }
  __syncthreads();
  const int p_hi = PART == 2 ? sp.n_wb - 1 : sp.P - 1;
  const int p_lo = PART == 1 ? sp.n_wb : 0;
  for (int p = p_hi; p >= p_lo; --p) {
    const bool wb = PART == 1 ? false : p < sp.n_wb;
    const int N = sp.N[p], ko = sp.ko[p];
    if (p + 1 < sp.P) {
      if constexpr (PART != 1) {
        if (wb) impact_step<NT>(sp, d, b, sh, lane, p, px_reads);
      }
      if (lane == 0) sh.dV = st->dV[p + 1];  // dVnext
    }
    __syncthreads();
    const real* pos = d.refpos + (size_t)b * sp.NK + ko;
    real* Gp = d.G + ((size_t)b * sp.NK + ko + N - 1) * 14;
    const real* xe = traj_ptr(sp, d, b, nom, ko + N - 1);
    int64_t kn = 0;
    bool ok;
    if constexpr (PART != 1) {
      if (wb) {
        terminal_value<NT, 14>(sp, st, sh, lane, p, pos[N - 1], xe, Gp);
        const int mode = sp.mode[p];
        ok = (mode == 1 || mode == 3) ? sweep_wb_phase<NT, true>(sp, d, b, st, sh, lane, p, reg, &kn)
                                      : sweep_wb_phase<NT, false>(sp, d, b, st, sh, lane, p, reg, &kn);
        *knots_wb += kn;
      }
    }
    if (!wb) {
      terminal_value<NT, 6>(sp, st, sh, lane, p, pos[N - 1], xe, Gp);
      ok = sweep_fb_phase<NT>(sp, d, b, st, sh, lane, p, reg, &kn);
    }
    *knots += kn;
    __syncthreads();
    if (lane == 0) st->dV[p] = sh.dV;
    __syncthreads();
    if (!ok) return false;
  }
  return true;
}

// WAVES: minimum resident waves per SIMD requested from the register allocator.  One wave
// per problem; while the batch fits one wave per SIMD (B <= 4 x CUs) the 1-wave build (no
// register cap, widest ILP) is fastest, beyond that the 2-wave build hides latency by
// co-residency.
//
// PART 0: the whole sweep with its regularisation retries (MultiPhaseDDP.cpp:196-241).
// PART 1: the SRB phases of the first attempt only, the value function at the WB boundary
// saved to d.carry.  PART 2: the WB phases of the first attempt (if PART 1 passed), then the
// same retries as PART 0 (whole sweeps) -- the same attempts with the same regularisation.
template <int NT, int WAVES, int PART>
__global__ __launch_bounds__(NT, WAVES) void k_bws(SolveParams sp, DevBufs d, real update_reg) {
  const int b = blockIdx.x;
  if (b >= sp.B) return;
  ProbState* st = &d.st[b];
  if (!(st->active && st->ddp_active)) return;
  __shared__ BwsLds sh;
  real reg = st->reg;
  int bws_iter = 1;
  int64_t knots = 0, knots_wb = 0, px_reads = 0, sweeps = 0;
  bool aborted = false;
  if constexpr (PART == 1) {
    const bool ok = bws_sweep<NT, 1>(sp, d, b, st, sh, reg, &knots, &knots_wb, &px_reads);
    BwsCarry& c = d.carry[b];
    #pragma unroll 1
    for (int e = threadIdx.x; e < 196; e += NT) c.H[e] = sh.H[e];
    if (threadIdx.x < 14) c.G[threadIdx.x] = sh.G[threadIdx.x];
    if (threadIdx.x == 0) {
      c.ok = ok ? 1 : 0;
      c.knots = (int32_t)knots;
    }
    return;
  }
  if constexpr (PART == 2) {
    // PART 0's loop below, the SRB half of its first attempt taken from PART 1; every
    // retry runs both halves here (one call site each: the WB sweep code exists once)
    const BwsCarry& c = d.carry[b];
    knots = c.knots;
    for (bool first = true;; first = false) {
      ++sweeps;
      bool ok = first ? c.ok != 0
                      : bws_sweep<NT, 1>(sp, d, b, st, sh, reg, &knots, &knots_wb, &px_reads);
      if (ok) ok = bws_sweep<NT, 2>(sp, d, b, st, sh, reg, &knots, &knots_wb, &px_reads, first);
      if (ok) break;
      reg = fmax(reg * update_reg, real(1e-03));  // MultiPhaseDDP.cpp:218
      ++bws_iter;
      if (reg > 1000) { aborted = true; break; }
    }
  }
#ifdef MHPC_BWS_TIMING
  if (threadIdx.x < 12) sh.cyc[threadIdx.x] = 0;
  if (threadIdx.x == 0) sh.tlast = clock64();
  const unsigned long long t_start = clock64();
  __syncthreads();
#endif
  if constexpr (PART == 0) {
    for (;;) {
      ++sweeps;
      if (bws_sweep<NT, 0>(sp, d, b, st, sh, reg, &knots, &knots_wb, &px_reads)) break;
      reg = fmax(reg * update_reg, real(1e-03));  // MultiPhaseDDP.cpp:218
      ++bws_iter;
      if (reg > 1000) { aborted = true; break; }
    }
  }
  __syncthreads();
#ifdef MHPC_BWS_TIMING
  if (threadIdx.x == 0) sh.cyc[0] = clock64() - t_start;
  __syncthreads();
  if (threadIdx.x < 12) atomicAdd(&g_bws_cyc[threadIdx.x], sh.cyc[threadIdx.x]);
#endif
  if (threadIdx.x == 0) {
    st->cnt[C_DDP]++;
    st->cnt[C_BWS] += sweeps;
    st->cnt[C_BWS_KNOTS] += knots;
    st->cnt[C_BWS_KNOTS_WB] += knots_wb;
    st->cnt[C_BWS_KNOTS_FB] += knots - knots_wb;
    st->cnt[C_PX_READS] += px_reads;
    if (PART == 2) st->cnt[C_BWS_KNOTS_FB1] += d.carry[b].knots;
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
      reg = reg / 20;          // MultiPhaseDDP.cpp:237-241
      if (reg < real(1e-06)) reg = 0;
      st->reg = reg;
    }
  }
}

// Variant: sp.var_bws (mhpc_set_kernel_variant) or, by default by batch size on the
// handle's device (sp.ncu CUs, 4 SIMDs each): two waves per problem (128-thread block, the
// WB rounds' products split over twice the lanes: -20 % cycles per WB knot) while both fit
// one SIMD each, the 1-wave build while one wave per problem does, the 2-wave (256-VGPR)
// build beyond.  All builds compile the same source; tests/test_gpu_variants.py checks them
// bit for bit.  The SRB half of a split sweep always runs 64-thread blocks (its rounds are
// narrower than a wave).
// part: 0 whole sweep, 1 / 2 its SRB / WB halves (bws_split).  The SRB half reads no
// partials record and needs few registers (the WB code is not instantiated), so a partials
// wave fits beside it on a SIMD.
// Waves per SIMD the register allocator targets in the beyond-one-wave-per-SIMD build.
#ifndef MHPC_BWS_MW
#define MHPC_BWS_MW 2
#endif
hipError_t launch_bws(const SolveParams& sp, const DevBufs& d, real update_reg, int part,
                      hipStream_t s) {
#ifdef MHPC_BWS_WAVES
  hipLaunchKernelGGL((k_bws<MHPC_BWS_NT, MHPC_BWS_WAVES, 0>), dim3(sp.B), dim3(MHPC_BWS_NT), 0, s,
                     sp, d, update_reg);
  (void)part;
#else
  const int v = sp.var_bws ? sp.var_bws
                           : sp.B <= 2 * sp.ncu ? MHPC_VARIANT_BWS_PAIRWAVE
                           : sp.B <= 4 * sp.ncu ? MHPC_VARIANT_BWS_1WAVE
                                                : MHPC_VARIANT_BWS_2WAVE;
  if (part == 1)
    hipLaunchKernelGGL((k_bws<64, 2, 1>), dim3(sp.B), dim3(64), 0, s, sp, d, update_reg);
  else if (v == MHPC_VARIANT_BWS_PAIRWAVE && part == 2)
    hipLaunchKernelGGL((k_bws<128, 1, 2>), dim3(sp.B), dim3(128), 0, s, sp, d, update_reg);
  else if (v == MHPC_VARIANT_BWS_1WAVE && part == 2)
    hipLaunchKernelGGL((k_bws<64, 1, 2>), dim3(sp.B), dim3(64), 0, s, sp, d, update_reg);
  else if (v == MHPC_VARIANT_BWS_2WAVE && part == 2)
    hipLaunchKernelGGL((k_bws<64, MHPC_BWS_MW, 2>), dim3(sp.B), dim3(64), 0, s, sp, d, update_reg);
  else if (v == MHPC_VARIANT_BWS_1WAVE)
    hipLaunchKernelGGL((k_bws<64, 1, 0>), dim3(sp.B), dim3(64), 0, s, sp, d, update_reg);
  else if (v == MHPC_VARIANT_BWS_2WAVE)
    hipLaunchKernelGGL((k_bws<64, MHPC_BWS_MW, 0>), dim3(sp.B), dim3(64), 0, s, sp, d, update_reg);
  else
    hipLaunchKernelGGL((k_bws<128, 1, 0>), dim3(sp.B), dim3(128), 0, s, sp, d, update_reg);
#endif
  return hipGetLastError();
}

// Whether the sweep runs as an SRB launch beside the partials and a WB launch after them:
// both kinds of phase present, not switched off (var_overlap 2).
bool bws_split(const SolveParams& sp) {
  return sp.n_wb > 0 && sp.P > sp.n_wb && sp.var_overlap != 2;
}

}  // namespace MHPC_NS

#ifdef MHPC_BWS_TIMING
extern "C" int mhpc_dbg_bws_cycles(unsigned long long* out, int reset) {
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(MHPC_NS::g_bws_cyc), sizeof(unsigned long long) * 12) !=
      hipSuccess)
    return 1;
  if (reset) {
    unsigned long long z[12] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(MHPC_NS::g_bws_cyc), z, sizeof(z)) != hipSuccess) return 1;
  }
  return 0;
}
#endif
