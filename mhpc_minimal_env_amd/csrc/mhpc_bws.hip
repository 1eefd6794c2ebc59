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

#include "mhpc_device.h"

namespace mhpc {

struct BwsLds {
  double H[196], G[14];  // value function of knot k+1, then of knot k (row stride NX)
  double W[7 * 18];      // rows NQ..NX-1 of [A B], stride NR = NX + 4
  double G2[2 * 18];     // stance rows of [C D]
  double l[18];          // (lx, lu)
  double lxx[14], luu[4];
  double lyy2[4], ly2[2];
  union {
    struct {
      double Jt[18 * 14];  // [A B]' H   (NR x NX)
      double Q[18 * 18];   // Qxx (NX x NX), Qux (rows NX.., cols ..NX), Quu (4x4), stride NR
    };
    struct {
      double H2[196];      // impact-aware step: lifted H' and (Px' H2)
      double Px[196];
      double T[196];
    };
  };
  double Qv[18];         // (Qx, Qu)
  double Qi[16], inv[16];
  double tq[14 * 4 + 16];  // Qux' Quu_inv (NX x 4) + scratch for the raw inverse
  double xb[14], ub[4], yb[4];
  double hx[14], Hs[9], G2v[14];
  double dV;
  int fail;
};

// Eigen-style 4x4 inverse by cofactors (same formulas as the oracle).
__device__ __forceinline__ void inverse4(const double* m, double* inv) {
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

// Symmetric swap of indices K < I of a 4x4 lower triangle, exactly as Eigen's
// ldlt_inplace<Lower>::unblocked applies a transposition (compile-time indices).
template <int K, int I>
__device__ __forceinline__ void ldlt_swap(double* A) {
#pragma unroll
  for (int j = 0; j < K; ++j) { const double t = A[K * 4 + j]; A[K * 4 + j] = A[I * 4 + j]; A[I * 4 + j] = t; }
#pragma unroll
  for (int i = I + 1; i < 4; ++i) { const double t = A[i * 4 + K]; A[i * 4 + K] = A[i * 4 + I]; A[i * 4 + I] = t; }
  { const double t = A[K * 4 + K]; A[K * 4 + K] = A[I * 4 + I]; A[I * 4 + I] = t; }
#pragma unroll
  for (int i = K + 1; i < I; ++i) { const double t = A[i * 4 + K]; A[i * 4 + K] = A[I * 4 + i]; A[I * 4 + i] = t; }
}

template <int K>
__device__ __forceinline__ void ldlt_pivot(double* A) {
  int big = K;
  double bv = fabs(A[K * 4 + K]);
#pragma unroll
  for (int i = K + 1; i < 4; ++i)
    if (fabs(A[i * 4 + i]) > bv) { bv = fabs(A[i * 4 + i]); big = i; }
  if (K < 1 && big == 1) ldlt_swap<(K < 1 ? K : 0), 1>(A);
  if (K < 2 && big == 2) ldlt_swap<(K < 2 ? K : 0), 2>(A);
  if (K < 3 && big == 3) ldlt_swap<(K < 3 ? K : 0), 3>(A);
}

// Eigen::LDLT(Quu - 1e-9 I).isPositive() (SinglePhase.cpp:202-209): diagonal pivoting,
// sign bookkeeping from ZeroSign; true iff no strictly negative pivot.
__device__ __forceinline__ bool ldlt_is_positive4(double* A) {
  int sign = 0;  // 0 ZeroSign, 1 PositiveSemiDef, 2 NegativeSemiDef, 3 Indefinite
  bool stop = false;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (stop) continue;
    if (k == 0) ldlt_pivot<0>(A);
    else if (k == 1) ldlt_pivot<1>(A);
    else if (k == 2) ldlt_pivot<2>(A);
    else ldlt_pivot<3>(A);
    if (k > 0) {
      double temp[3];
#pragma unroll
      for (int j = 0; j < k; ++j) temp[j] = A[j * 4 + j] * A[k * 4 + j];
      double s = 0;
#pragma unroll
      for (int j = 0; j < k; ++j) s += A[k * 4 + j] * temp[j];
      A[k * 4 + k] -= s;
#pragma unroll
      for (int i = k + 1; i < 4; ++i) {
        double t = 0;
#pragma unroll
        for (int j = 0; j < k; ++j) t += A[i * 4 + j] * temp[j];
        A[i * 4 + k] -= t;
      }
    }
    const double akk = A[k * 4 + k];
    const bool valid = fabs(akk) > 0.0;
    if (k == 0 && !valid) { sign = 0; stop = true; continue; }
    if (k < 3 && valid) {
#pragma unroll
      for (int i = k + 1; i < 4; ++i) A[i * 4 + k] /= akk;
    }
    if (sign == 1) { if (akk < 0.0) sign = 3; }
    else if (sign == 2) { if (akk > 0.0) sign = 3; }
    else if (sign == 0) { if (akk > 0.0) sign = 1; else if (akk < 0.0) sign = 2; }
  }
  return sign == 1 || sign == 0;
}

// Row coefficient of the exact part of [A B] (see file header).
template <int NQ>
__device__ __forceinline__ double coef_a(int col, double dt) {
  return col < NQ ? 1.0 : (col < 2 * NQ ? dt : 0.0);
}
template <int NQ>
__device__ __forceinline__ int coef_b(int col) {
  return col < NQ ? col : col - NQ;
}

// One Riccati knot.  On entry sh.{W,G2,l,lxx,luu,lyy2,ly2} hold the knot's derivatives and
// sh.{H,G} the value function of knot k+1; on exit sh.{H,G} hold that of knot k.
#ifndef MHPC_BWS_CH2
#define MHPC_BWS_CH2 3
#endif
#ifndef MHPC_BWS_CH3
#define MHPC_BWS_CH3 3
#endif
#ifndef MHPC_BWS_CH5
#define MHPC_BWS_CH5 4
#endif
constexpr int CH2 = MHPC_BWS_CH2, CH3 = MHPC_BWS_CH3, CH5 = MHPC_BWS_CH5;

template <int NQ, bool HAS_Y>
__device__ bool riccati_knot(BwsLds& sh, int lane, double dt, double reg, double eps9,
                             double* Kout, double* duout, double* Gout) {
  constexpr int NX = 2 * NQ, NR = NX + 4;
  // R2: Jt = [A B]' H (NR x NX) and Qv = (l + [A B]' G) + [C D]' ly.
  // Lane = (column j of H, row group g): the column H[NQ.., j] stays in registers and the
  // lane runs up to RPL independent row chains (ILP); the last QL lanes build Qv.
  {
    constexpr int QL = NX == 14 ? 8 : 10;     // lanes for Qv
    constexpr int G = (64 - QL) / NX;          // row groups
    constexpr int RPL = (NR + G - 1) / G;      // rows per lane
    if (lane < G * NX) {
      const int j = lane % NX, g = lane / NX;
      double hc[NQ];
#pragma unroll
      for (int r = 0; r < NQ; ++r) hc[r] = sh.H[(NQ + r) * NX + j];
      constexpr int C = RPL < CH2 ? RPL : CH2;  // chains in flight
#pragma unroll 1
      for (int t0 = 0; t0 < RPL; t0 += C) {
        double acc[C];
#pragma unroll
        for (int u = 0; u < C; ++u) {
          const int row = g + G * (t0 + u);
          double sacc = 0.0;
          if (row < NR) {
            const double a = coef_a<NQ>(row, dt);
            if (a != 0.0) sacc = a * sh.H[coef_b<NQ>(row) * NX + j];
#pragma unroll
            for (int r = 0; r < NQ; ++r) sacc += sh.W[r * NR + row] * hc[r];
          }
          acc[u] = sacc;
        }
#pragma unroll
        for (int u = 0; u < C; ++u) {
          const int row = g + G * (t0 + u);
          if (row < NR) sh.Jt[row * NX + j] = acc[u];
        }
      }
    } else {
      const int q = lane - G * NX;
      double gc[NQ];
#pragma unroll
      for (int r = 0; r < NQ; ++r) gc[r] = sh.G[NQ + r];
#pragma unroll
      for (int t = 0; t < (NR + QL - 1) / QL; ++t) {
        const int row = q + QL * t;
        if (row < NR) {
          const double a = coef_a<NQ>(row, dt);
          double sacc = 0.0, tt = 0.0;
          if (a != 0.0) sacc = a * sh.G[coef_b<NQ>(row)];
#pragma unroll
          for (int r = 0; r < NQ; ++r) sacc += sh.W[r * NR + row] * gc[r];
          if (HAS_Y) tt = sh.G2[row] * sh.ly2[0] + sh.G2[NR + row] * sh.ly2[1];
          sh.Qv[row] = (sh.l[row] + sacc) + tt;
        }
      }
    }
  }
  __syncthreads();
  // R3: Qxx = (lxx + C'lyy C) + A'HA ; Qux = (0 + D'lyy C) + B'HA ; Quu = (luu + D'lyy D) + B'HB
  // Lane = (row of Jt, column group g): the row Jt[row, NQ..] stays in registers, up to CPL
  // independent column chains per lane.
  {
    constexpr int RG = 64 / NR;                    // column groups
    constexpr int CPL = (NR + RG - 1) / RG;        // columns per lane
    if (lane < RG * NR) {
      const int row = lane % NR, g = lane / NR;
      const int ncol = row < NX ? NX : NR;
      double jr[NQ];
#pragma unroll
      for (int r = 0; r < NQ; ++r) jr[r] = sh.Jt[row * NX + NQ + r];
      double gr0 = 0.0, gr1 = 0.0, c0 = 0.0, c1 = 0.0;
      if (HAS_Y) {
        gr0 = sh.G2[row];
        gr1 = sh.G2[NR + row];
        c0 = gr0 * sh.lyy2[0] + gr1 * sh.lyy2[2];
        c1 = gr0 * sh.lyy2[1] + gr1 * sh.lyy2[3];
      }
      constexpr int C = CPL < CH3 ? CPL : CH3;
#pragma unroll 1
      for (int t0 = 0; t0 < CPL; t0 += C) {
        double acc[C];
#pragma unroll
        for (int u = 0; u < C; ++u) {
          const int col = g + RG * (t0 + u);
          double v = 0.0;
          if (col < ncol) {
            const double a = coef_a<NQ>(col, dt);
            double sacc = 0.0;
            if (a != 0.0) sacc = a * sh.Jt[row * NX + coef_b<NQ>(col)];
#pragma unroll
            for (int r = 0; r < NQ; ++r) sacc += jr[r] * sh.W[r * NR + col];
            double base = 0.0;
            if (row == col) base = row < NX ? sh.lxx[row] : sh.luu[row - NX];
            double e2 = 0.0;
            if (HAS_Y) e2 = c0 * sh.G2[col] + c1 * sh.G2[NR + col];
            v = (base + e2) + sacc;
            if (row == col) v += 1.0 * reg;
          }
          acc[u] = v;
        }
#pragma unroll
        for (int u = 0; u < C; ++u) {
          const int col = g + RG * (t0 + u);
          if (col < ncol) sh.Q[row * NR + col] = acc[u];
        }
      }
    }
  }
  __syncthreads();
  // R4: PSD test of Quu - 1e-9 I (every lane, registers, static indices), then the
  // adjugate of Quu spread over lanes 0..15 (one 3x3 minor each)
  {
    double A[16];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        A[i * 4 + c] = sh.Q[(NX + i) * NR + NX + c] - (i == c ? 1.0 * eps9 : 0.0);
    if (!ldlt_is_positive4(A)) return false;
  }
  if (lane < 16) {
    // adj[i][j] = (-1)^(i+j) det(minor without row j, column i)
    const int i = lane >> 2, j = lane & 3;
    const int r0 = j == 0 ? 1 : 0, r1 = j <= 1 ? 2 : 1, r2 = j <= 2 ? 3 : 2;
    const int c0 = i == 0 ? 1 : 0, c1 = i <= 1 ? 2 : 1, c2 = i <= 2 ? 3 : 2;
    const double* q = &sh.Q[NX * NR + NX];
#define QM(r, c) q[(r) * NR + (c)]
    const double det3 = QM(r0, c0) * (QM(r1, c1) * QM(r2, c2) - QM(r1, c2) * QM(r2, c1)) -
                        QM(r0, c1) * (QM(r1, c0) * QM(r2, c2) - QM(r1, c2) * QM(r2, c0)) +
                        QM(r0, c2) * (QM(r1, c0) * QM(r2, c1) - QM(r1, c1) * QM(r2, c0));
#undef QM
    sh.inv[lane] = ((i + j) & 1) ? -det3 : det3;
  }
  __syncthreads();
  if (lane < 16) {
    const double* q = &sh.Q[NX * NR + NX];
    const double det = q[0] * sh.inv[0] + q[1] * sh.inv[4] + q[2] * sh.inv[8] + q[3] * sh.inv[12];
    const int t = ((lane & 3) << 2) | (lane >> 2);
    const double a = sh.inv[lane] / det, at = sh.inv[t] / det;
    sh.Qi[lane] = (a + at) / 2;  // Quu_inv = (inv + inv')/2
    sh.tq[4 * NX + lane] = a;    // unsymmetrised inverse, for dV
  }
  __syncthreads();
  // R4b: K = -Quu_inv Qux, tq = Qux' Quu_inv, du = -Quu_inv Qu, dV = -Qu' Quu^-1 Qu
  if (lane == 63) {
    double s = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      double t = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) t += sh.Qv[NX + k] * sh.tq[4 * NX + k * 4 + c];
      s += t * sh.Qv[NX + c];
    }
    sh.dV += -s;  // unsymmetrised inverse, no 1/2 (MHPC_CompoundTypes.h:142)
  }
  __syncthreads();
  #pragma unroll 1
  for (int e = lane; e < 8 * NX + 4; e += 64) {
    if (e < 4 * NX) {
      const int c = e / NX, j = e - c * NX;
      double s = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) s += -sh.Qi[c * 4 + k] * sh.Q[(NX + k) * NR + j];
      Kout[c * NX + j] = s;
    } else if (e < 8 * NX) {
      const int q = e - 4 * NX, i = q >> 2, c = q & 3;
      double s = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) s += sh.Q[(NX + k) * NR + i] * sh.Qi[k * 4 + c];
      sh.tq[q] = s;
    } else {
      const int c = e - 8 * NX;
      double s = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) s += -sh.Qi[c * 4 + k] * sh.Qv[NX + k];
      duout[c] = s;
    }
  }
  __syncthreads();
  // R5: H = sym(Qxx) - tq Qux ; G = Qx - tq Qu.  Lane = (column j, row group): the column
  // Qux[., j] stays in registers, up to 4 independent row chains per lane.
  {
    constexpr int G5 = 56 / NX;               // 4 for NX = 14, 9 for NX = 6
    constexpr int R5 = (NX + G5 - 1) / G5;
    if (lane < G5 * NX) {
      const int j = lane % NX, g = lane / NX;
      double qc[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) qc[c] = sh.Q[(NX + c) * NR + j];
      constexpr int C = R5 < CH5 ? R5 : CH5;
#pragma unroll 1
      for (int t0 = 0; t0 < R5; t0 += C) {
        double acc[C];
#pragma unroll
        for (int u = 0; u < C; ++u) {
          const int i = g + G5 * (t0 + u);
          double v = 0.0;
          if (i < NX) {
            double sacc = 0;
#pragma unroll
            for (int c = 0; c < 4; ++c) sacc += sh.tq[i * 4 + c] * qc[c];
            v = (sh.Q[i * NR + j] + sh.Q[j * NR + i]) / 2 - sacc;
          }
          acc[u] = v;
        }
#pragma unroll
        for (int u = 0; u < C; ++u) {
          const int i = g + G5 * (t0 + u);
          if (i < NX) sh.H[i * NX + j] = acc[u];
        }
      }
    } else {
      for (int i = lane - G5 * NX; i < NX; i += 64 - G5 * NX) {
        double sacc = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) sacc += sh.tq[i * 4 + c] * sh.Qv[NX + c];
        const double gi = sh.Qv[i] - sacc;
        sh.G[i] = gi;
        Gout[i] = gi;
      }
    }
  }
  __syncthreads();
  return true;
}

// Running-cost derivatives of a WB knot: lx / lxx per state lane (CostBase.cpp:28-31),
// the control / force part comes precomputed with the partials record (see mhpc_solver.h).
__device__ __forceinline__ void wb_cost_x(BwsLds& sh, int lane, const SolveParams& sp, double dt,
                                          double pos) {
  if (lane < 14) {
    const int i = lane;
    const double rxi = i == 0 ? pos : i == 1 ? sp.height : i == 2 ? 0.0
                       : i < 7 ? cQjointBias[i - 3] : i == 7 ? sp.vel : 0.0;
    sh.l[i] = (2 * dt * cQwb[i]) * (sh.xb[i] - rxi);
    sh.lxx[i] = 2 * dt * cQwb[i];
  }
}

// SRB Jacobian entry of row 3+r, column col of [A B] (FBDynamics_par.c operation order).
__device__ __forceinline__ double srb_w_entry(int r, int col, const double* x, const double* u,
                                              const double* p, const double* s, double dt) {
  MHPC_NO_FMA
  const int row = 3 + r;
  double ac = 0.0;
  if (col < 6) {
    if (row == 5 && col == 0) ac = s[0] * (kSrbInvInertia * u[1]) + s[1] * (kSrbInvInertia * u[3]);
    if (row == 5 && col == 1) ac = -(s[0] * (kSrbInvInertia * u[0]) + s[1] * (kSrbInvInertia * u[2]));
    return (col == row ? 1.0 : 0.0) + ac * dt;
  }
  const int c = col - 6;
  double bc = 0.0;
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
template <int NX>
__device__ void terminal_value(const SolveParams& sp, const ProbState* st, BwsLds& sh, int lane,
                               int p, double pos, const double* xe, double* Gout) {
  constexpr bool wb = NX == 14;
  const int mode = sp.mode[p];
  const bool al = wb && ntc_of(mode, true) && sp.AL_active && st->al_partials;
  double h = 0;
  if (al && lane == 0) {
    double hx[14], Hs[3][3];
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
  const double s = st->sigma[p], lam = st->lambda[p];
  const int ih = mode == 2 ? 3 : 5;  // touchdown Hessian block (theta, hip, knee)
  #pragma unroll 1
  for (int e = lane; e < NX * NX + NX; e += 64) {
    if (e < NX * NX) {
      const int i = e / NX, j = e - i * NX;
      double v = i == j ? (wb ? cQfwb[mode - 1][i] : cQffb[i]) : 0.0;
      if (al) {
        const int ai = i == 2 ? 0 : (i == ih ? 1 : (i == ih + 1 ? 2 : -1));
        const int aj = j == 2 ? 0 : (j == ih ? 1 : (j == ih + 1 ? 2 : -1));
        const double hij = (ai >= 0 && aj >= 0) ? sh.Hs[ai * 3 + aj] : 0.0;
        v += 50 * (s * s / 2 * (sh.hx[i] * sh.hx[j] + h * hij) + lam * hij);
      }
      sh.H[e] = v + sh.H[e];
    } else {
      const int i = e - NX * NX;
      double rxi;
      if (wb) rxi = i == 0 ? pos : (i == 7 ? sp.vel : cXtermWB[mode - 1][i]);
      else rxi = i == 0 ? pos : (i == 1 ? sp.height : (i == 3 ? sp.vel : 0.0));
      double v = (wb ? cQfwb[mode - 1][i] : cQffb[i]) * (xe[i] - rxi);
      if (al) v += 50 * (s * s / 2 * sh.hx[i] * h + lam * sh.hx[i]);
      const double g = v + sh.G[i];
      sh.G[i] = g;
      Gout[i] = g;
    }
  }
  __syncthreads();
}

// impact_aware_step (MultiPhaseDDP.cpp:300-341) for a WB phase p: sh.G/H hold CTG[0] of
// phase p+1 (6-dim if that phase is SRB); on exit the 14-dim Gnext/Hnext of phase p.
__device__ void impact_step(const SolveParams& sp, const DevBufs& d, int b, BwsLds& sh, int lane,
                            int p, int64_t* px_reads) {
  const int mode = sp.mode[p];
  const bool nwb = p + 1 < sp.n_wb;
  const bool imp = mode == 2 || mode == 4;
  // lift to the full-model space: E' G', E' H' E (E = _stateProj for an SRB next phase)
  #pragma unroll 1
  for (int e = lane; e < 196 + 14; e += 64) {
    if (e < 196) {
      const int i = e / 14, j = e - i * 14;
      double v;
      if (nwb) v = sh.H[e];
      else {
        const int pi = i < 3 ? i : (i >= 7 && i < 10 ? i - 4 : -1);
        const int pj = j < 3 ? j : (j >= 7 && j < 10 ? j - 4 : -1);
        v = (pi >= 0 && pj >= 0) ? sh.H[pi * 6 + pj] : 0.0;
      }
      sh.H2[e] = v;
    } else {
      const int i = e - 196;
      double v;
      if (nwb) v = sh.G[i];
      else {
        const int q = i < 3 ? i : (i >= 7 && i < 10 ? i - 4 : -1);
        v = q >= 0 ? sh.G[q] : 0.0;
      }
      sh.G2v[i] = v;
    }
  }
  if (imp) {
    const double* pxc = d.px + ((size_t)b * MAXP + p) * 196;  // column-major
    #pragma unroll 1
    for (int e = lane; e < 196; e += 64) sh.Px[(e % 14) * 14 + e / 14] = pxc[e];
    if (lane == 0) ++*px_reads;
  }
  __syncthreads();
  if (imp) {
    // G = Px' G2 ; T = Px' H2 ; H = T Px
    #pragma unroll 1
    for (int e = lane; e < 196 + 14; e += 64) {
      if (e < 196) {
        const int i = e / 14, j = e - i * 14;
        double s = 0;
#pragma unroll
        for (int m = 0; m < 14; ++m) s += sh.Px[m * 14 + i] * sh.H2[m * 14 + j];
        sh.T[e] = s;
      } else {
        const int i = e - 196;
        double s = 0;
#pragma unroll
        for (int m = 0; m < 14; ++m) s += sh.Px[m * 14 + i] * sh.G2v[m];
        sh.G[i] = s;
      }
    }
    __syncthreads();
    #pragma unroll 1
    for (int e = lane; e < 196; e += 64) {
      const int i = e / 14, j = e - i * 14;
      double s = 0;
#pragma unroll
      for (int m = 0; m < 14; ++m) s += sh.T[i * 14 + m] * sh.Px[m * 14 + j];
      sh.H[e] = s;
    }
  } else {
    #pragma unroll 1
    for (int e = lane; e < 196; e += 64) sh.H[e] = sh.H2[e];
    if (lane < 14) sh.G[lane] = sh.G2v[lane];
  }
  __syncthreads();
}

// Backward sweep of one WB phase: knots N-2..0 with a one-knot register prefetch.
__device__ bool sweep_wb_phase(const SolveParams& sp, const DevBufs& d, int b, const ProbState* st,
                               BwsLds& sh, int lane, int p, double reg, int64_t* knots) {
  const int N = sp.N[p], ko = sp.ko[p], mode = sp.mode[p];
  const double dt = sp.dt[p];
  const int nom = st->nom_slot;
  const bool stance = mode == 1 || mode == 3;
  const double* pos = d.refpos + (size_t)b * sp.NK + ko;
  constexpr int NR = 18;
  // prefetch registers: 3 doubles of the partials record + 1 of the nominal knot
  double pre[3], prex = 0;
  auto load = [&](int k) {
    const double* prec = d.par + ((size_t)b * sp.NK + ko + k) * PS;
#pragma unroll
    for (int t = 0; t < 3; ++t) {  // 3 x 64 lanes >= PS = 176
      const int e = lane + 64 * t;
      pre[t] = e < PS ? prec[e] : 0.0;
    }
    if (lane < 22) prex = traj_ptr(sp, d, b, nom, ko + k)[lane];
  };
  load(N - 2);
  for (int k = N - 2; k >= 0; --k) {
    const int kk = ko + k;
    // drop the prefetched knot into LDS: W = rows 7..13 of [I + dt Ac | dt Bc], G2 = [C D]
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int e = lane + 64 * t;
      if (e < PS_JAC) {
        const int col = e / 9, r = e - col * 9;
        if (r < 7) sh.W[r * NR + col] = (col == 7 + r ? 1.0 : 0.0) + pre[t] * dt;
        else if (stance) sh.G2[(r - 7) * NR + col] = pre[t];
      } else if (e < PS) {
        const int q = e - PS_JAC;  // lu 4, luu 4, ly 2, lyy 4
        if (q < 4) sh.l[14 + q] = pre[t];
        else if (q < 8) sh.luu[q - 4] = pre[t];
        else if (q < 10) sh.ly2[q - 8] = pre[t];
        else sh.lyy2[q - 10] = pre[t];
      }
    }
    if (lane < 14) sh.xb[lane] = prex;
    else if (lane < 18) sh.ub[lane - 14] = prex;
    else if (lane < 22) sh.yb[lane - 18] = prex;
    __syncthreads();
    if (k > 0) load(k - 1);
    wb_cost_x(sh, lane, sp, dt, pos[k]);
    __syncthreads();
    double* Kout = d.K + ((size_t)b * sp.NK + kk) * 56;
    double* duout = d.du + ((size_t)b * sp.NK + kk) * 4;
    double* Gout = d.G + ((size_t)b * sp.NK + kk) * 14;
    const bool ok = stance
                        ? riccati_knot<7, true>(sh, lane, dt, reg, sp.eps9, Kout, duout, Gout)
                        : riccati_knot<7, false>(sh, lane, dt, reg, sp.eps9, Kout, duout, Gout);
    ++*knots;
    if (!ok) return false;
  }
  return true;
}

__device__ bool sweep_fb_phase(const SolveParams& sp, const DevBufs& d, int b, const ProbState* st,
                               BwsLds& sh, int lane, int p, double reg, int64_t* knots) {
  const int N = sp.N[p], ko = sp.ko[p], mode = sp.mode[p];
  const double dt = sp.dt[p];
  const int nom = st->nom_slot;
  const double* pos = d.refpos + (size_t)b * sp.NK + ko;
  constexpr int NR = 10;
  double foot[4], cs[2];
  plan_foothold(traj_ptr(sp, d, b, nom, ko), dt * N, mode, foot);
  srb_contact(mode, cs);
  const int m = mode - 1;
  double prex = 0;
  if (lane < 10) prex = traj_ptr(sp, d, b, nom, ko + N - 2)[lane];
  for (int k = N - 2; k >= 0; --k) {
    const int kk = ko + k;
    if (lane < 6) sh.xb[lane] = prex;
    else if (lane < 10) sh.ub[lane - 6] = prex;
    __syncthreads();
    if (k > 0 && lane < 10) prex = traj_ptr(sp, d, b, nom, ko + k - 1)[lane];
    if (lane < 30) {
      const int r = lane / 10, col = lane - r * 10;
      sh.W[r * NR + col] = srb_w_entry(r, col, sh.xb, sh.ub, foot, cs, dt);
    } else if (lane < 36) {
      const int i = lane - 30;
      const double rxi = i == 0 ? pos[k] : i == 1 ? sp.height : i == 3 ? sp.vel : 0.0;
      sh.l[i] = (2 * dt * cQfb[i]) * (sh.xb[i] - rxi);
      sh.lxx[i] = 2 * dt * cQfb[i];
    } else if (lane < 40) {
      const int c = lane - 36;
      const double ru = (c == 1 || c == 3) ? 8.252 * 9.81 : 0.0;
      sh.l[6 + c] = (2 * dt * cRfb[m][c]) * (sh.ub[c] - ru);
      sh.luu[c] = 2 * dt * cRfb[m][c];
    }
    __syncthreads();
    double* Kout = d.K + ((size_t)b * sp.NK + kk) * 56;
    double* duout = d.du + ((size_t)b * sp.NK + kk) * 4;
    double* Gout = d.G + ((size_t)b * sp.NK + kk) * 14;
    const bool ok = riccati_knot<3, false>(sh, lane, dt, reg, sp.eps9, Kout, duout, Gout);
    ++*knots;
    if (!ok) return false;
  }
  return true;
}

__device__ bool bws_sweep(const SolveParams& sp, const DevBufs& d, int b, ProbState* st, BwsLds& sh,
                          double reg, int64_t* knots, int64_t* knots_wb, int64_t* px_reads) {
  const int lane = threadIdx.x;
  const int nom = st->nom_slot;
  #pragma unroll 1
  for (int e = lane; e < 196; e += 64) sh.H[e] = 0;  // Gnext = 0, Hnext = 0 (last phase)
  if (lane < 14) sh.G[lane] = 0;
  if (lane == 0) sh.dV = 0;
  __syncthreads();
  for (int p = sp.P - 1; p >= 0; --p) {
    const bool wb = p < sp.n_wb;
    const int N = sp.N[p], ko = sp.ko[p];
    if (p + 1 < sp.P) {
      if (wb) impact_step(sp, d, b, sh, lane, p, px_reads);
      if (lane == 0) sh.dV = st->dV[p + 1];  // dVnext
    }
    __syncthreads();
    const double* pos = d.refpos + (size_t)b * sp.NK + ko;
    double* Gp = d.G + ((size_t)b * sp.NK + ko + N - 1) * 14;
    const double* xe = traj_ptr(sp, d, b, nom, ko + N - 1);
    int64_t kn = 0;
    bool ok;
    if (wb) {
      terminal_value<14>(sp, st, sh, lane, p, pos[N - 1], xe, Gp);
      ok = sweep_wb_phase(sp, d, b, st, sh, lane, p, reg, &kn);
      *knots_wb += kn;
    } else {
      terminal_value<6>(sp, st, sh, lane, p, pos[N - 1], xe, Gp);
      ok = sweep_fb_phase(sp, d, b, st, sh, lane, p, reg, &kn);
    }
    *knots += kn;
    __syncthreads();
    if (lane == 0) st->dV[p] = sh.dV;
    __syncthreads();
    if (!ok) return false;
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
  int64_t knots = 0, knots_wb = 0, px_reads = 0, sweeps = 0;
  bool aborted = false;
  for (;;) {
    ++sweeps;
    if (bws_sweep(sp, d, b, st, sh, reg, &knots, &knots_wb, &px_reads)) break;
    reg = fmax(reg * update_reg, 1e-03);  // MultiPhaseDDP.cpp:218
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
      if (reg < 1e-06) reg = 0;
      st->reg = reg;
    }
  }
}

hipError_t launch_bws(const SolveParams& sp, const DevBufs& d, double update_reg, hipStream_t s) {
  hipLaunchKernelGGL(k_bws, dim3(sp.B), dim3(64), 0, s, sp, d, update_reg);
  return hipGetLastError();
}

}  // namespace mhpc
