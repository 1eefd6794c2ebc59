// Hand-written planar-quadruped physics for the MHPC solve path.
//
// Replaces, as device code, every CasADi-generated kernel the reference calls on its
// HSDDP path:
//   Dyn_FL / Dyn_BS / Dyn_FS      -> wb_dynamics()          (PlanarQuadruped.cpp:8-27)
//   Dyn_*_par                     -> wb_dynamics<Dual>()    (PlanarQuadruped.cpp:30-53)
//   Imp_F / Imp_B (+ _par)        -> wb_impact()            (PlanarQuadruped.cpp:58-100)
//   WB_FL1/FL2_terminal_constr    -> wb_touchdown()         (MHPCConstraints.cpp:91-107)
//   Jacob_F / Jacob_B             -> wb_foot_jacobian()     (PlanarQuadruped.cpp:103-117)
//   FBDynamics / FBDynamics_par   -> srb_dynamics(), srb_jacobians() (PlanarFloatingBase.cpp:7-72)
//
// Model: q = (x, z, theta, q_fhip, q_fknee, q_bhip, q_bknee),
// x = (q, qdot), u = torques on the four leg joints.  A point a distance l "down" a link
// whose absolute angle is a sits at (-l sin a, -l cos a) from that link's joint; the
// front/back hips sit at (x +- 0.19 cos th, z -+ 0.19 sin th).  M(q) and the bias
// h(q, qdot) are assembled body by body from CoM Jacobians (M = sum m Jc'Jc + Ic w w',
// h = sum m Jc'(Jcdot qdot + g)), which is exact for a planar tree.  Stance and impact
// solve the contact KKT system through the Schur complement J M^-1 J' of a block-arrowhead
// factorisation of M (the reference's generated code uses an unpivoted QR instead; both agree
// to ~1e-12, see tests/test_model_host.py).
//
// Everything is templated on the scalar so the same source runs in real (rollouts)
// and in Dual (one Jacobian column per lane).
//
// No FMA contraction in the whole-body functions below (MHPC_NO_FMA): the line search's
// lane-pair model (mhpc_model_pair.h) forms each leg's terms on its own lane and sums them
// after a lane swap, where a product cannot fuse into the sum; with every product rounded
// in both models the result depends only on the order of operations, which the two share,
// so they agree bit for bit (tests/test_gpu_kernels.py::test_wb_dynamics_pair_bitwise,
// tests/test_pair_host.py) and a problem's result does not depend on which line-search
// variant its batch size selects.
#pragma once
#include <type_traits>
#include "mhpc_dual.h"

// MHPC_WB_FMA (timing experiments only) lets the compiler contract the whole-body model
// again; the line-search variants then no longer agree bit for bit.
#ifdef MHPC_WB_FMA
#define MHPC_NO_FMA_WB
#else
#define MHPC_NO_FMA_WB MHPC_NO_FMA
#endif

namespace MHPC_NS {

// ---- parameters baked into the reference's generated code ----------
constexpr real kGrav = real(9.81);
constexpr real kBodyMass = real(5.46);
constexpr real kBodyInertia = real(0.116419);        // about the body CoM
constexpr real kHipX = real(0.19);                   // hip joints at +-0.19 on the body axis
constexpr real kThighMass = real(1.268);
constexpr real kThighCom = real(0.02);               // CoM distance down the thigh
constexpr real kThighInertiaJoint = real(0.0047132); // about the hip joint
constexpr real kThighLen = real(0.209);              // hip -> knee
constexpr real kShankMass = real(0.128);
constexpr real kShankCom = real(0.061);
constexpr real kShankInertiaJoint = real(0.000972288);  // about the knee joint
constexpr real kShankLen = real(0.195);              // knee -> foot
constexpr real kGroundHeight = -real(0.404);         // MHPCLocomotion.cpp:25, WB_FL*_terminal_constr.c
constexpr real kThighInertiaCom = kThighInertiaJoint - kThighMass * kThighCom * kThighCom;
constexpr real kShankInertiaCom = kShankInertiaJoint - kShankMass * kShankCom * kShankCom;

// SRB constants (FBDynamics.c:51-100): total mass and pitch inertia of the floating base.
constexpr real kSrbMass = real(8.2520000000000007);
constexpr real kSrbInertia = real(0.23216549759999999);
constexpr real kSrbInvInertia = real(4.3072722275163766);  // as folded by FBDynamics_par.c
constexpr real kSrbInvMass = real(1.2118274357731458e-01);

constexpr int kWbX = 14, kWbQ = 7, kWbU = 4, kWbY = 4;
constexpr int kFbX = 6, kFbU = 4, kFbY = 4;

enum Foot { kFront = 0, kBack = 1 };

// Two scalar types run through the model: Q for everything that depends on the
// configuration q only (link sines/cosines, Jacobians, M and its factorisation) and V for
// what also depends on qdot or u (link rates, bias h, Jdot qdot, accelerations, forces).
// Q = V = real is the plain model; Q = V = Dual differentiates along a q direction; Q =
// real, V = Dual differentiates along a qdot or u direction, where M, its factorisation
// and the Jacobians carry exactly zero derivative -- the same numbers at a fraction of the
// work (the Jacobian pass, k_partials).

// Geometry of one leg: absolute link angles and their sines/cosines.
template <class Q, class V>
struct LegGeo {
  Q s1, c1, s2, c2;  // thigh angle a1 = th + q_hip, shank angle a2 = a1 + q_knee
  V w1, w2;          // absolute angular rates
};

template <class Q, class V>
struct WbGeo {
  Q sth, cth;           // body pitch
  LegGeo<Q, V> leg[2];  // [front, back]
};

// xq = q (7), xv = qdot (7)
// BATCH: the real-valued angles through sin_cos_n (fewer instructions; more live registers,
// so the register-bound partials keep the one-at-a-time form).  Same values either way.
template <class Q, class V, bool BATCH = true>
MHPC_HD void wb_geometry(const Q* xq, const V* xv, WbGeo<Q, V>& g, const SinCosK& K = kSinCosK) {
  if constexpr (BATCH && std::is_same<Q, real>::value) {
    // the five link angles' sines / cosines side by side (sin_cos_n)
    const real a[5] = {xq[2], xq[2] + xq[3], (xq[2] + xq[3]) + xq[4], xq[2] + xq[5],
                       (xq[2] + xq[5]) + xq[6]};
    real sv[5], cv[5];
    sin_cos_n<5>(a, sv, cv, K);
    g.sth = sv[0]; g.cth = cv[0];
    g.leg[0].s1 = sv[1]; g.leg[0].c1 = cv[1]; g.leg[0].s2 = sv[2]; g.leg[0].c2 = cv[2];
    g.leg[1].s1 = sv[3]; g.leg[1].c1 = cv[3]; g.leg[1].s2 = sv[4]; g.leg[1].c2 = cv[4];
  } else {
    (void)K;
    sin_cos(xq[2], &g.sth, &g.cth);
    for (int f = 0; f < 2; ++f) {
      const int ih = 3 + 2 * f, ik = 4 + 2 * f;
      const Q a1 = xq[2] + xq[ih];
      const Q a2 = a1 + xq[ik];
      sin_cos(a1, &g.leg[f].s1, &g.leg[f].c1);
      sin_cos(a2, &g.leg[f].s2, &g.leg[f].c2);
    }
  }
  for (int f = 0; f < 2; ++f) {
    const int ih = 3 + 2 * f, ik = 4 + 2 * f;
    g.leg[f].w1 = xv[2] + xv[ih];
    g.leg[f].w2 = g.leg[f].w1 + xv[ik];
  }
}

// Jacobian of a point on leg F at distance l1 down the thigh and l2 down the shank,
// compact over the local columns (x, z, th, hip, knee), plus the centripetal part of
// Jdot*qdot due to the two link rotations (the hip-offset part is added by the caller).
// The leg index is a template parameter everywhere so that no register array is indexed
// with a run-time value (which would spill it to scratch memory on the GPU).
template <class Q, class V, int F>
MHPC_HD void leg_point_jac(const WbGeo<Q, V>& g, real l1, real l2, Q jx[5], Q jz[5], V* jdx,
                           V* jdz) {
  MHPC_NO_FMA_WB
  constexpr real sg = F == kFront ? real(1.0) : -real(1.0);
  const LegGeo<Q, V>& L = g.leg[F];
  // d/da of l*(-sin a, -cos a) = l*(-cos a, sin a)
  const Q tx1 = -l1 * L.c1, tz1 = l1 * L.s1;
  const Q tx2 = -l2 * L.c2, tz2 = l2 * L.s2;
  jx[0] = Q(real(1.0)); jz[0] = Q(real(0.0));
  jx[1] = Q(real(0.0)); jz[1] = Q(real(1.0));
  jx[4] = tx2;    jz[4] = tz2;
  jx[3] = tx1 + tx2;
  jz[3] = tz1 + tz2;
  jx[2] = mad(-sg * kHipX, g.sth, jx[3]);
  jz[2] = mad(-sg * kHipX, g.cth, jz[3]);
  *jdx = mad(L.w1 * L.w1, l1 * L.s1, L.w2 * L.w2 * (l2 * L.s2));
  *jdz = mad(L.w1 * L.w1, l1 * L.c1, L.w2 * L.w2 * (l2 * L.c2));
}

// Packed lower-triangular index of the symmetric 7x7 mass matrix.
MHPC_HD constexpr int tri(int i, int j) { return i * (i + 1) / 2 + j; }

// Contribution of the thigh and shank of leg F to M (packed) and h.  xv = qdot.  The
// entries shared with the other leg -- M(2, 0..2) and h(0..2) -- are returned per leg as
// thigh + shank (bm, bh) and summed by the caller as front + back: a sum of two terms is
// the same whichever lane of the line search's lane pair holds which (mhpc_model_pair.h).
template <class Q, class V, int F>
MHPC_HD void add_leg(const V* xv, const WbGeo<Q, V>& g, Q M[28], V h[7], Q bm[3], V bh[3]) {
  MHPC_NO_FMA_WB
  constexpr real sg = F == kFront ? real(1.0) : -real(1.0);
  constexpr int idx[5] = {0, 1, 2, 3 + 2 * F, 4 + 2 * F};
  const V thd2 = xv[2] * xv[2];
  const V hax = (-sg * kHipX) * g.cth * thd2;  // centripetal acceleration of the hip point
  const V haz = (sg * kHipX) * g.sth * thd2;
#pragma unroll
  for (int b = 0; b < 2; ++b) {  // thigh, shank
    Q jx[5], jz[5];
    V jdx, jdz;
    real m, ic;
    if (b == 0) {
      leg_point_jac<Q, V, F>(g, kThighCom, real(0.0), jx, jz, &jdx, &jdz);
      m = kThighMass; ic = kThighInertiaCom;
    } else {
      leg_point_jac<Q, V, F>(g, kThighLen, kShankCom, jx, jz, &jdx, &jdz);
      m = kShankMass; ic = kShankInertiaCom;
    }
    const int nc = b == 0 ? 4 : 5;
    jdx += hax;
    jdz += haz;
    const V ax = jdx, az = jdz + kGrav;
#pragma unroll
    for (int a = 0; a < 5; ++a) {
      if (a >= nc) continue;
      const V dh = m * mad(jx[a], ax, jz[a] * az);
      if (a < 3) bh[a] = b == 0 ? dh : bh[a] + dh;
      else h[idx[a]] += dh;
#pragma unroll
      for (int c = 0; c <= a; ++c) {
        // x/z columns of a CoM Jacobian are unit vectors: skip the exact zeros
        if (a < 2 && c < 2) {
          if (a == c) M[tri(idx[a], idx[c])] += Q(m);
          continue;
        }
        Q v = m * mad(jx[a], jx[c], jz[a] * jz[c]);
        if (a >= 2 && c >= 2) v += ic;
        if (a == 2) bm[c] = b == 0 ? v : bm[c] + v;
        else M[tri(idx[a], idx[c])] += v;
      }
    }
  }
}

// M(q) (packed lower triangle, 28 entries) and bias h(q, qdot) = C qdot + g.
template <class Q, class V>
MHPC_HD void wb_mass_bias(const V* xv, const WbGeo<Q, V>& g, Q M[28], V h[7]) {
#pragma unroll
  for (int i = 0; i < 7; ++i) h[i] = V(real(0.0));
#pragma unroll
  for (int i = 0; i < 28; ++i) M[i] = Q(real(0.0));
  M[tri(0, 0)] = Q(kBodyMass);
  M[tri(1, 1)] = Q(kBodyMass);
  Q bmf[3], bmb[3];
  V bhf[3], bhb[3];
  add_leg<Q, V, kFront>(xv, g, M, h, bmf, bhf);
  add_leg<Q, V, kBack>(xv, g, M, h, bmb, bhb);
  // shared entries: constant + (front + back)
  const real m2[3] = {real(0.0), real(0.0), kBodyInertia};
  const real h0[3] = {real(0.0), kBodyMass * kGrav, real(0.0)};
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    M[tri(2, c)] = Q(m2[c]) + (bmf[c] + bmb[c]);
    h[c] = V(h0[c]) + (bhf[c] + bhb[c]);
  }
}

// Block-arrowhead factorisation of the mass matrix.  Ordered (base x,z,th | front leg |
// back leg), M has no front/back-leg coupling, so it is solved by eliminating the two 2x2
// leg blocks first and factoring the 3x3 base Schur complement S (no fill-in, three
// reciprocals, no square roots) -- the tree structure an articulated-body solver exploits.
template <class S>
struct ArrowFactor {
  S Li[2][3];   // inverse of each 2x2 leg block (a, b, c of [[a b][b c]]^-1)
  S Z[2][2][3]; // Z_l = Ml^-1 * M_lb  (2 x 3)
  S Si[6];      // inverse of the base Schur complement, packed symmetric (00,10,11,20,21,22)
};

template <class S>
MHPC_HD void arrow_factor(const S M[28], ArrowFactor<S>& F) {
  MHPC_NO_FMA_WB
  // base Schur complement S = Mbb - sum_l Mlb' Ml^-1 Mlb (symmetric, lower packed)
  S s00 = M[tri(0, 0)], s10 = M[tri(1, 0)], s11 = M[tri(1, 1)];
  S s20 = M[tri(2, 0)], s21 = M[tri(2, 1)], s22 = M[tri(2, 2)];
  S t[2][6];
#pragma unroll
  for (int l = 0; l < 2; ++l) {
    const int i0 = 3 + 2 * l, i1 = 4 + 2 * l;
    const S a = M[tri(i0, i0)], b = M[tri(i1, i0)], c = M[tri(i1, i1)];
    const S rdet = pivot_rcp(mad(a, c, -(b * b)));
    F.Li[l][0] = c * rdet;
    F.Li[l][1] = -b * rdet;
    F.Li[l][2] = a * rdet;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const S m0 = M[tri(i0, j)], m1 = M[tri(i1, j)];
      F.Z[l][0][j] = mad(F.Li[l][0], m0, F.Li[l][1] * m1);
      F.Z[l][1][j] = mad(F.Li[l][1], m0, F.Li[l][2] * m1);
    }
    // leg l's term of S -= sum_l Mlb' Z_l
    const S* z0 = F.Z[l][0];
    const S* z1 = F.Z[l][1];
    t[l][0] = mad(M[tri(i0, 0)], z0[0], M[tri(i1, 0)] * z1[0]);
    t[l][1] = mad(M[tri(i0, 1)], z0[0], M[tri(i1, 1)] * z1[0]);
    t[l][2] = mad(M[tri(i0, 1)], z0[1], M[tri(i1, 1)] * z1[1]);
    t[l][3] = mad(M[tri(i0, 2)], z0[0], M[tri(i1, 2)] * z1[0]);
    t[l][4] = mad(M[tri(i0, 2)], z0[1], M[tri(i1, 2)] * z1[1]);
    t[l][5] = mad(M[tri(i0, 2)], z0[2], M[tri(i1, 2)] * z1[2]);
  }
  // front + back (see add_leg)
  s00 -= t[0][0] + t[1][0];
  s10 -= t[0][1] + t[1][1];
  s11 -= t[0][2] + t[1][2];
  s20 -= t[0][3] + t[1][3];
  s21 -= t[0][4] + t[1][4];
  s22 -= t[0][5] + t[1][5];
  // 3x3 symmetric inverse by cofactors
  const S c00 = mad(s11, s22, -(s21 * s21));
  const S c10 = mad(s21, s20, -(s10 * s22));
  const S c20 = mad(s10, s21, -(s11 * s20));
  const S rdet = pivot_rcp(mad(s20, c20, mad(s10, c10, s00 * c00)));
  F.Si[0] = c00 * rdet;
  F.Si[1] = c10 * rdet;
  F.Si[2] = mad(s00, s22, -(s20 * s20)) * rdet;
  F.Si[3] = c20 * rdet;
  F.Si[4] = mad(s20, s10, -(s00 * s21)) * rdet;
  F.Si[5] = mad(s00, s11, -(s10 * s10)) * rdet;
}

// b <- M^-1 b  (M, factor in Q; b in V)
template <class Q, class V>
MHPC_HD void arrow_solve(const Q M[28], const ArrowFactor<Q>& F, V b[7]) {
  MHPC_NO_FMA_WB
  V w[2][2], t[2][3];
#pragma unroll
  for (int l = 0; l < 2; ++l) {
    const int i0 = 3 + 2 * l, i1 = 4 + 2 * l;
    w[l][0] = mad(F.Li[l][0], b[i0], F.Li[l][1] * b[i1]);
    w[l][1] = mad(F.Li[l][1], b[i0], F.Li[l][2] * b[i1]);
    t[l][0] = mad(M[tri(i0, 0)], w[l][0], M[tri(i1, 0)] * w[l][1]);
    t[l][1] = mad(M[tri(i0, 1)], w[l][0], M[tri(i1, 1)] * w[l][1]);
    t[l][2] = mad(M[tri(i0, 2)], w[l][0], M[tri(i1, 2)] * w[l][1]);
  }
  // base rows minus front + back (see add_leg)
  const V r0 = b[0] - (t[0][0] + t[1][0]);
  const V r1 = b[1] - (t[0][1] + t[1][1]);
  const V r2 = b[2] - (t[0][2] + t[1][2]);
  const V x0 = mad(F.Si[3], r2, mad(F.Si[1], r1, F.Si[0] * r0));
  const V x1 = mad(F.Si[4], r2, mad(F.Si[2], r1, F.Si[1] * r0));
  const V x2 = mad(F.Si[5], r2, mad(F.Si[4], r1, F.Si[3] * r0));
  b[0] = x0;
  b[1] = x1;
  b[2] = x2;
#pragma unroll
  for (int l = 0; l < 2; ++l) {
    b[3 + 2 * l] = w[l][0] - mad(F.Z[l][0][2], x2, mad(F.Z[l][0][1], x1, F.Z[l][0][0] * x0));
    b[4 + 2 * l] = w[l][1] - mad(F.Z[l][1][2], x2, mad(F.Z[l][1][1], x1, F.Z[l][1][0] * x0));
  }
}

// Foot Jacobian (2x7, dense) and Jdot*qdot of foot F.  xv = qdot.
template <class Q, class V, int F>
MHPC_HD void wb_foot_jac_full(const V* xv, const WbGeo<Q, V>& g, Q J[2][7], V jd[2]) {
  MHPC_NO_FMA_WB
  Q jx[5], jz[5];
  V jdx, jdz;
  leg_point_jac<Q, V, F>(g, kThighLen, kShankLen, jx, jz, &jdx, &jdz);
  constexpr real sg = F == kFront ? real(1.0) : -real(1.0);
  const V thd2 = xv[2] * xv[2];
  jd[0] = jdx + (-sg * kHipX) * g.cth * thd2;
  jd[1] = jdz + (sg * kHipX) * g.sth * thd2;
  constexpr int idx[5] = {0, 1, 2, 3 + 2 * F, 4 + 2 * F};
#pragma unroll
  for (int i = 0; i < 7; ++i) { J[0][i] = Q(real(0.0)); J[1][i] = Q(real(0.0)); }
#pragma unroll
  for (int a = 0; a < 5; ++a) { J[0][idx[a]] = jx[a]; J[1][idx[a]] = jz[a]; }
}

// Schur-complement solve of the contact KKT system
//   [M -J'; J 0] [v; lam] = [rhs; -c]  ->  v = M^-1 (rhs + J' lam)
// given the factorisation of M; v holds M^-1 rhs on entry.
template <class Q, class V>
MHPC_HD void kkt_contact(const Q M[28], const ArrowFactor<Q>& F, const Q J[2][7], const V c[2],
                         V v[7], V lam[2]) {
  MHPC_NO_FMA_WB
  Q Y[2][7];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
#pragma unroll
    for (int i = 0; i < 7; ++i) Y[r][i] = J[r][i];
    arrow_solve<Q, Q>(M, F, Y[r]);
  }
  Q A00 = Q(real(0.0)), A01 = Q(real(0.0)), A11 = Q(real(0.0));
  V r0 = -c[0], r1 = -c[1];
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    A00 = mad(J[0][i], Y[0][i], A00);
    A01 = mad(J[0][i], Y[1][i], A01);
    A11 = mad(J[1][i], Y[1][i], A11);
    r0 = mad(-J[0][i], v[i], r0);
    r1 = mad(-J[1][i], v[i], r1);
  }
  const Q rdet = pivot_rcp(mad(A00, A11, -(A01 * A01)));
  lam[0] = mad(A11, r0, -(A01 * r1)) * rdet;
  lam[1] = mad(A00, r1, -(A01 * r0)) * rdet;
#pragma unroll
  for (int i = 0; i < 7; ++i) v[i] += mad(Y[0][i], lam[0], Y[1][i] * lam[1]);
}

// Stance dynamics with foot F on the ground (Dyn_FS: F = front, Dyn_BS: F = back).
template <class Q, class V, int F>
MHPC_HD void wb_stance(const V* xv, const WbGeo<Q, V>& g, const Q M[28],
                       const ArrowFactor<Q>& AF, V v[7], V* y) {
  Q J[2][7];
  V jd[2], lam[2];
  wb_foot_jac_full<Q, V, F>(xv, g, J, jd);
  kkt_contact<Q, V>(M, AF, J, jd, v, lam);
  y[2 * F] = lam[0];
  y[2 * F + 1] = lam[1];
}

// Continuous whole-body dynamics with q in Q and (qdot, u) in V: xdot = (qdot, qddot),
// y = contact force of the stance foot in its slots (front -> y[0:2], back -> y[2:4]);
// zero in flight.  mode 1: back stance (Dyn_BS), 2/4: flight (Dyn_FL), 3: front stance
// (Dyn_FS).
template <class Q, class V>
MHPC_HD void wb_dynamics_qv(const Q* xq, const V* xv, const V* u, int mode, V* xdot, V* y,
                            const SinCosK& K = kSinCosK) {
  WbGeo<Q, V> g;
  wb_geometry<Q, V>(xq, xv, g, K);
  Q M[28];
  V h[7];
  wb_mass_bias<Q, V>(xv, g, M, h);
  ArrowFactor<Q> AF;
  arrow_factor(M, AF);
  V v[7];
  v[0] = -h[0]; v[1] = -h[1]; v[2] = -h[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) v[3 + i] = u[i] - h[3 + i];
  arrow_solve<Q, V>(M, AF, v);
#pragma unroll
  for (int i = 0; i < 4; ++i) y[i] = V(real(0.0));
  if (mode == 1) wb_stance<Q, V, kBack>(xv, g, M, AF, v, y);
  else if (mode == 3) wb_stance<Q, V, kFront>(xv, g, M, AF, v, y);
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    xdot[i] = xv[i];
    xdot[7 + i] = v[i];
  }
}

// The plain interface: x = (q, qdot) in one scalar type.
template <class S>
MHPC_HD void wb_dynamics(const S* x, const S* u, int mode, S* xdot, S* y, const SinCosK& K = kSinCosK) {
  wb_dynamics_qv<S, S>(x, x + 7, u, mode, xdot, y, K);
}

// ---- Jacobians by implicit differentiation (the partials kernel, Dyn_*_par) --------------
// The forward dynamics solve the contact KKT system
//   R = M(q) qdd + h(q, qd) - S'u - J(q)' lam = 0,   C = J(q) qdd + Jd(q, qd) qd = 0
// (C and lam only in stance).  Along a direction th of (q, qd, u), with qdd and lam held at
// the knot's solution,  [M -J'; J 0] [dqdd; dlam] = -[R_th; C_th]:  one dual-number
// evaluation of the residuals (inverse dynamics -- no factorisation, no division, the link
// sines / cosines of the knot reused) and a solve with the knot's own factorisation, instead
// of a dual-number evaluation of the whole forward dynamics per direction.  Same derivative
// as forward-mode differentiation of wb_dynamics up to rounding.
struct WbKnot {
  WbGeo<real, real> g;
  real M[28];              // packed mass matrix (the solves read its leg coupling rows)
  ArrowFactor<real> AF;
  real qdd[7], lam[2];
  real J[2][7];            // stance foot Jacobian (stance only)
  real A00, A01, A11, rdet;  // J M^-1 J' and 1 / its determinant (stance only)
};

// The knot's forward dynamics (wb_dynamics' arithmetic), keeping what the solves reuse.
// SF: stance foot (kFront: mode 3, kBack: mode 1) or -1 (flight, modes 2 and 4).
template <int SF>
MHPC_HD void wb_knot_primal(const real* x, const real* u, WbKnot& K) {
  MHPC_NO_FMA_WB
  wb_geometry<real, real, false>(x, x + 7, K.g);
  real h[7], v[7];
  wb_mass_bias<real, real>(x + 7, K.g, K.M, h);
  arrow_factor(K.M, K.AF);
  v[0] = -h[0]; v[1] = -h[1]; v[2] = -h[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) v[3 + i] = u[i] - h[3 + i];
  arrow_solve<real, real>(K.M, K.AF, v);
  K.lam[0] = K.lam[1] = real(0.0);
  if constexpr (SF >= 0) {
    real jd[2];
    wb_foot_jac_full<real, real, SF>(x + 7, K.g, K.J, jd);
    real Y[2][7];  // M^-1 J'
#pragma unroll
    for (int r = 0; r < 2; ++r) {
#pragma unroll
      for (int i = 0; i < 7; ++i) Y[r][i] = K.J[r][i];
      arrow_solve<real, real>(K.M, K.AF, Y[r]);
    }
    real A00 = real(0.0), A01 = real(0.0), A11 = real(0.0), r0 = -jd[0], r1 = -jd[1];
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      A00 = mad(K.J[0][i], Y[0][i], A00);
      A01 = mad(K.J[0][i], Y[1][i], A01);
      A11 = mad(K.J[1][i], Y[1][i], A11);
      r0 = mad(-K.J[0][i], v[i], r0);
      r1 = mad(-K.J[1][i], v[i], r1);
    }
    K.A00 = A00; K.A01 = A01; K.A11 = A11;
    K.rdet = pivot_rcp(mad(A00, A11, -(A01 * A01)));
    K.lam[0] = mad(A11, r0, -(A01 * r1)) * K.rdet;
    K.lam[1] = mad(A00, r1, -(A01 * r0)) * K.rdet;
#pragma unroll
    for (int i = 0; i < 7; ++i) v[i] += mad(Y[0][i], K.lam[0], Y[1][i] * K.lam[1]);
  }
#pragma unroll
  for (int i = 0; i < 7; ++i) K.qdd[i] = v[i];
}

// [M -J'; J 0] [v; lam] = [rhs; -c] with the knot's factorisation (rhs in v on entry);
// out = (v 7, lam 2) -- one column of the partials record.  The contact correction
// M^-1 J' lam is a second arrow solve rather than M^-1 J' kept per knot (14 fewer live
// doubles per lane).
template <int SF>
MHPC_HD void wb_knot_solve(const WbKnot& K, real v[7], real c0, real c1, real out[9]) {
  MHPC_NO_FMA_WB
  arrow_solve<real, real>(K.M, K.AF, v);
  real l0 = real(0.0), l1 = real(0.0);
  if constexpr (SF >= 0) {
    real r0 = -c0, r1 = -c1;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      r0 = mad(-K.J[0][i], v[i], r0);
      r1 = mad(-K.J[1][i], v[i], r1);
    }
    l0 = mad(K.A11, r0, -(K.A01 * r1)) * K.rdet;
    l1 = mad(K.A00, r1, -(K.A01 * r0)) * K.rdet;
    real w[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) w[i] = mad(K.J[0][i], l0, K.J[1][i] * l1);
    arrow_solve<real, real>(K.M, K.AF, w);
#pragma unroll
    for (int i = 0; i < 7; ++i) v[i] += w[i];
  }
#pragma unroll
  for (int i = 0; i < 7; ++i) out[i] = v[i];
  out[7] = l0;
  out[8] = l1;
}

// Inverse dynamics of leg F's thigh and shank at the fixed qdd: adds
// m Jc'(Jc qdd + Jcdot qd + g) + Ic w (w . qdd) of each body to R (add_leg's M qdd + h).
template <class Q, class V, int F>
MHPC_HD void id_leg(const V* xv, const WbGeo<Q, V>& g, const real* qdd, V R[7]) {
  MHPC_NO_FMA_WB
  constexpr real sg = F == kFront ? real(1.0) : -real(1.0);
  constexpr int idx[5] = {0, 1, 2, 3 + 2 * F, 4 + 2 * F};
  const V thd2 = xv[2] * xv[2];
  const V hax = (-sg * kHipX) * g.cth * thd2;
  const V haz = (sg * kHipX) * g.sth * thd2;
  const real al1 = qdd[2] + qdd[idx[3]];  // angular accelerations of thigh and shank
  const real al2 = al1 + qdd[idx[4]];
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    Q jx[5], jz[5];
    V jdx, jdz;
    real m, ic;
    if (b == 0) {
      leg_point_jac<Q, V, F>(g, kThighCom, real(0.0), jx, jz, &jdx, &jdz);
      m = kThighMass; ic = kThighInertiaCom;
    } else {
      leg_point_jac<Q, V, F>(g, kThighLen, kShankCom, jx, jz, &jdx, &jdz);
      m = kShankMass; ic = kShankInertiaCom;
    }
    const int nc = b == 0 ? 4 : 5;
    // CoM acceleration (x/z columns of Jc are unit vectors)
    V ax = (jdx + hax) + qdd[0], az = ((jdz + haz) + kGrav) + qdd[1];
#pragma unroll
    for (int a = 2; a < 5; ++a) {
      if (a >= nc) continue;
      ax = mad(jx[a], qdd[idx[a]], ax);
      az = mad(jz[a], qdd[idx[a]], az);
    }
    const real ia = ic * (b == 0 ? al1 : al2);
    R[0] += m * ax;
    R[1] += m * az;
#pragma unroll
    for (int a = 2; a < 5; ++a) {
      if (a >= nc) continue;
      R[idx[a]] += m * mad(jx[a], ax, jz[a] * az) + ia;
    }
  }
}

// Tangents of R and C along one direction, given the link geometry g in (Q, V) (the body
// terms of M qdd + h and the stance foot's J' lam, C = J qdd + Jd qd; the constant base
// terms and S'u carry no tangent).
template <class Q, class V, int SF>
MHPC_HD void wb_residual_tangent(const V* xv, const WbGeo<Q, V>& g, const WbKnot& K, real rhs[7],
                                 real* c0, real* c1) {
  MHPC_NO_FMA_WB
  V R[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) R[i] = V(real(0.0));
  id_leg<Q, V, kFront>(xv, g, K.qdd, R);
  id_leg<Q, V, kBack>(xv, g, K.qdd, R);
  *c0 = *c1 = real(0.0);
  if constexpr (SF >= 0) {
    Q jx[5], jz[5];
    V jdx, jdz;
    leg_point_jac<Q, V, SF>(g, kThighLen, kShankLen, jx, jz, &jdx, &jdz);
    constexpr real sg = SF == kFront ? real(1.0) : -real(1.0);
    constexpr int idx[5] = {0, 1, 2, 3 + 2 * SF, 4 + 2 * SF};
    const V thd2 = xv[2] * xv[2];
    V C0 = jdx + (-sg * kHipX) * g.cth * thd2;
    V C1 = jdz + (sg * kHipX) * g.sth * thd2;
    C0 = C0 + K.qdd[0];
    C1 = C1 + K.qdd[1];
#pragma unroll
    for (int a = 2; a < 5; ++a) {
      C0 = mad(jx[a], K.qdd[idx[a]], C0);
      C1 = mad(jz[a], K.qdd[idx[a]], C1);
    }
    R[0] -= V(K.lam[0]);
    R[1] -= V(K.lam[1]);
#pragma unroll
    for (int a = 2; a < 5; ++a) R[idx[a]] -= mad(jx[a], K.lam[0], jz[a] * K.lam[1]);
    *c0 = tangent(C0);
    *c1 = tangent(C1);
  }
#pragma unroll
  for (int i = 0; i < 7; ++i) rhs[i] = -tangent(R[i]);
}

// Column dir of the continuous Jacobians: d qdd (7) and d lam (2) of the stance foot.
// q directions (dir 0..6): dual geometry from the knot's sines / cosines.
template <int SF>
MHPC_HD void wb_knot_partial_q(const real* x, const WbKnot& K, int dir, real out[9]) {
  MHPC_NO_FMA_WB
  real rhs[7], c0, c1;
  const real dth = dir == 2 ? real(1.0) : real(0.0);
  WbGeo<Dual, Dual> g;
  g.sth = Dual(K.g.sth, K.g.cth * dth);
  g.cth = Dual(K.g.cth, -K.g.sth * dth);
  Dual xv[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) xv[i] = Dual(x[7 + i]);
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int ih = 3 + 2 * f, ik = 4 + 2 * f;
    const real d1 = dth + (dir == ih ? real(1.0) : real(0.0));
    const real d2 = d1 + (dir == ik ? real(1.0) : real(0.0));
    const LegGeo<real, real>& P = K.g.leg[f];
    g.leg[f].s1 = Dual(P.s1, P.c1 * d1);
    g.leg[f].c1 = Dual(P.c1, -P.s1 * d1);
    g.leg[f].s2 = Dual(P.s2, P.c2 * d2);
    g.leg[f].c2 = Dual(P.c2, -P.s2 * d2);
    g.leg[f].w1 = Dual(P.w1);
    g.leg[f].w2 = Dual(P.w2);
  }
  wb_residual_tangent<Dual, Dual, SF>(xv, g, K, rhs, &c0, &c1);
  wb_knot_solve<SF>(K, rhs, c0, c1, out);
}
// qd directions (dir 7..13): only the link rates carry a tangent (M, J: none).
template <int SF>
MHPC_HD void wb_knot_partial_qd(const real* x, const WbKnot& K, int dir, real out[9]) {
  MHPC_NO_FMA_WB
  real rhs[7], c0, c1;
  Dual xv[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) xv[i] = Dual(x[7 + i], 7 + i == dir ? real(1.0) : real(0.0));
  WbGeo<real, Dual> g;
  g.sth = K.g.sth;
  g.cth = K.g.cth;
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int ih = 3 + 2 * f, ik = 4 + 2 * f;
    g.leg[f].s1 = K.g.leg[f].s1; g.leg[f].c1 = K.g.leg[f].c1;
    g.leg[f].s2 = K.g.leg[f].s2; g.leg[f].c2 = K.g.leg[f].c2;
    g.leg[f].w1 = xv[2] + xv[ih];
    g.leg[f].w2 = g.leg[f].w1 + xv[ik];
  }
  wb_residual_tangent<real, Dual, SF>(xv, g, K, rhs, &c0, &c1);
  wb_knot_solve<SF>(K, rhs, c0, c1, out);
}
// u directions (dir 14..17): rhs = S'e, no constraint tangent.
template <int SF>
MHPC_HD void wb_knot_partial_u(const WbKnot& K, int dir, real out[9]) {
  real rhs[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) rhs[i] = 3 + (dir - 14) == i ? real(1.0) : real(0.0);
  wb_knot_solve<SF>(K, rhs, real(0.0), real(0.0), out);
}
template <int SF>
MHPC_HD void wb_knot_partial(const real* x, const WbKnot& K, int dir, real out[9]) {
  if (dir < 7) wb_knot_partial_q<SF>(x, K, dir, out);
  else if (dir < 14) wb_knot_partial_qd<SF>(x, K, dir, out);
  else wb_knot_partial_u<SF>(K, dir, out);
}

// One column (dir 0..13: Ac / C, 14..17: Bc / D) of the dense continuous Jacobians of
// Dyn_*_par by implicit differentiation: a (14 rows: the qd rows of xdot = (qd, qdd), then
// d qdd), c (4 rows of y, the stance foot's two).  For the eval hooks and host checks; the
// partials kernel writes the record directly.
template <int SF>
MHPC_HD void wb_partial_column_sf(const real* x, const real* u, int dir, real a[14], real c[4]) {
  WbKnot K;
  wb_knot_primal<SF>(x, u, K);
  real o[9];
  wb_knot_partial<SF>(x, K, dir, o);
  for (int i = 0; i < 7; ++i) {
    a[i] = dir == 7 + i ? real(1.0) : real(0.0);
    a[7 + i] = o[i];
  }
  for (int i = 0; i < 4; ++i) c[i] = real(0.0);
  if (SF >= 0) {
    c[2 * SF] = o[7];
    c[2 * SF + 1] = o[8];
  }
}
MHPC_HD void wb_partial_column(const real* x, const real* u, int mode, int dir, real a[14],
                               real c[4]) {
  if (mode == 1) wb_partial_column_sf<kBack>(x, u, dir, a, c);
  else if (mode == 3) wb_partial_column_sf<kFront>(x, u, dir, a, c);
  else wb_partial_column_sf<-1>(x, u, dir, a, c);
}

// Plastic impact of foot F (Imp_F: front, end of mode 2; Imp_B: back, end of mode 4):
// q+ = q, [M -J'; J 0][qd+; Lam] = [M qd-; 0].
template <class S, int F>
MHPC_HD void wb_impact_f(const S* x, S* xp, S* Lam) {
  MHPC_NO_FMA_F32
  WbGeo<S, S> g;
  wb_geometry<S, S>(x, x + 7, g);
  S M[28], h[7];
  wb_mass_bias<S, S>(x + 7, g, M, h);
  ArrowFactor<S> AF;
  arrow_factor(M, AF);
  S J[2][7], jd[2];
  wb_foot_jac_full<S, S, F>(x + 7, g, J, jd);
  S v[7], c[2];
#pragma unroll
  for (int i = 0; i < 7; ++i) v[i] = x[7 + i];  // M^-1 (M qd-) = qd-
  c[0] = S(real(0.0));
  c[1] = S(real(0.0));
  kkt_contact<S, S>(M, AF, J, c, v, Lam);  // J qd+ = 0
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    xp[i] = x[i];
    xp[7 + i] = v[i];
  }
}

template <class S>
MHPC_HD void wb_impact(const S* x, int f, S* xp, S* Lam) {
  if (f == kFront) wb_impact_f<S, kFront>(x, xp, Lam);
  else wb_impact_f<S, kBack>(x, xp, Lam);
}

// Touchdown constraint h = foot_z + 0.404 (foot F = front for mode 2 / WB_FL1, back for
// mode 4 / WB_FL2) with its gradient hx (14) and the 3x3 non-zero block of its Hessian on
// the state indices (theta, hip, knee) of that leg.
template <int F>
MHPC_HD real wb_touchdown_value(const real* x) {
  MHPC_NO_FMA_F32
  constexpr real sg = F == kFront ? real(1.0) : -real(1.0);
  constexpr int ih = 3 + 2 * F, ik = 4 + 2 * F;
  const real a1 = x[2] + x[ih];
  const real a2 = a1 + x[ik];
  return x[1] - sg * kHipX * sin(x[2]) - kThighLen * cos(a1) - kShankLen * cos(a2) - kGroundHeight;
}

template <int F>
MHPC_HD void wb_touchdown_compact(const real* x, real* h, real* hx, real Hs[3][3]) {
  constexpr real sg = F == kFront ? real(1.0) : -real(1.0);
  constexpr int ih = 3 + 2 * F, ik = 4 + 2 * F;
  real sth, cth, s1, c1, s2, c2;
  sin_cos(x[2], &sth, &cth);
  const real a1 = x[2] + x[ih];
  const real a2 = a1 + x[ik];
  sin_cos(a1, &s1, &c1);
  sin_cos(a2, &s2, &c2);
  *h = x[1] - sg * kHipX * sth - kThighLen * c1 - kShankLen * c2 - kGroundHeight;
#pragma unroll
  for (int i = 0; i < 14; ++i) hx[i] = real(0.0);
  const real dk = kShankLen * s2;
  const real dh = kThighLen * s1 + dk;
  hx[1] = real(1.0);
  hx[2] = -sg * kHipX * cth + dh;
  hx[ih] = dh;
  hx[ik] = dk;
  const real ek = kShankLen * c2;
  const real eh = kThighLen * c1 + ek;
  const real et = sg * kHipX * sth + eh;
  Hs[0][0] = et; Hs[0][1] = eh; Hs[0][2] = ek;
  Hs[1][0] = eh; Hs[1][1] = eh; Hs[1][2] = ek;
  Hs[2][0] = ek; Hs[2][1] = ek; Hs[2][2] = ek;
}

// Dense form (row-major 14x14 Hessian) used by host checks and the eval hooks.
MHPC_HD void wb_touchdown(const real* x, int f, real* h, real* hx, real* hxx) {
  real Hs[3][3];
  if (f == kFront) wb_touchdown_compact<kFront>(x, h, hx, Hs);
  else wb_touchdown_compact<kBack>(x, h, hx, Hs);
  const int id[3] = {2, 3 + 2 * f, 4 + 2 * f};
  for (int i = 0; i < 196; ++i) hxx[i] = real(0.0);
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b) hxx[id[a] * 14 + id[b]] = Hs[a][b];
}

// Foot Jacobian J (2x7, row-major) and Jdot (2x7) as used by the PD warm start
// (Jacob_F / Jacob_B; boundingPDControl.cpp:29,35).
template <int F>
MHPC_HD void wb_foot_jacobian_f(const real* x, real* J, real* Jd) {
  WbGeo<real, real> g;
  wb_geometry<real, real>(x, x + 7, g);
  real Jm[2][7], jd[2];
  wb_foot_jac_full<real, real, F>(x + 7, g, Jm, jd);
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int i = 0; i < 7; ++i) J[r * 7 + i] = Jm[r][i];
  constexpr real sg = F == kFront ? real(1.0) : -real(1.0);
  const LegGeo<real, real>& L = g.leg[F];
  const real thd = x[9];
#pragma unroll
  for (int i = 0; i < 14; ++i) Jd[i] = real(0.0);
  // d/dt of -l*cos a = l sin a * adot ; d/dt of l*sin a = l cos a * adot
  const real kx = kShankLen * L.s2 * L.w2, kz = kShankLen * L.c2 * L.w2;
  const real hx = kThighLen * L.s1 * L.w1 + kx, hz = kThighLen * L.c1 * L.w1 + kz;
  constexpr int ih = 3 + 2 * F, ik = 4 + 2 * F;
  Jd[0 * 7 + ik] = kx;  Jd[1 * 7 + ik] = kz;
  Jd[0 * 7 + ih] = hx;  Jd[1 * 7 + ih] = hz;
  Jd[0 * 7 + 2] = -sg * kHipX * g.cth * thd + hx;
  Jd[1 * 7 + 2] = sg * kHipX * g.sth * thd + hz;
}

MHPC_HD void wb_foot_jacobian(const real* x, int f, real* J, real* Jd) {
  if (f == kFront) wb_foot_jacobian_f<kFront>(x, J, Jd);
  else wb_foot_jacobian_f<kBack>(x, J, Jd);
}

// Hip-to-foot vector of leg F (PlanarQuadruped::get_leg_ext_vec, PlanarQuadruped.cpp:195-205).
template <int F>
MHPC_HD void wb_leg_ext(const real* q, real* v) {
  constexpr int ih = 3 + 2 * F, ik = 4 + 2 * F;
  real s1, c1, s2, c2;
  sin_cos(q[2] + q[ih], &s1, &c1);
  sin_cos(q[2] + q[ih] + q[ik], &s2, &c2);
  v[0] = -kThighLen * s1 - kShankLen * s2;
  v[1] = -kThighLen * c1 - kShankLen * c2;
}

// ---- single rigid body (PlanarFloatingBase + FBDynamics) ---------------------------
// x = (px, pz, th, vx, vz, w), u = (FFx, FFz, FBx, FBz), p = footholds (pFx, pFz, pBx,
// pBz), s = contact flags (front, back).  Operation order follows FBDynamics.c so the
// SRB arithmetic is bit-identical to the reference's.
MHPC_HD void srb_contact(int mode, real s[2]) {
  s[0] = mode == 3 ? real(1.0) : real(0.0);
  s[1] = mode == 1 ? real(1.0) : real(0.0);
}

// a / c for a positive constant c with rc = RN(1 / c), correctly rounded -- the IEEE
// quotient bit for bit for finite a (Markstein: q0 = RN(a rc) is within an ulp of a / c, the
// residual a - q0 c is exact in one FMA, and one correction step rounds correctly; sampled
// against IEEE division on 6e8 operands of both constants below, fp64 and fp32, no
// difference).  A zero residual keeps q0: exact, with the quotient's sign of zero.  Three
// dependent FP instructions instead of the division sequence (rcp + scale + 2 Newton steps +
// fixup), on every SRB knot of every rollout.
MHPC_HD real div_const(real a, real c, real rc) {
  const real q0 = a * rc;
  const real e = fma(-q0, c, a);
  const real q1 = fma(e, rc, q0);
  return e == real(0.0) ? q0 : q1;
}
constexpr real kSrbMassRcp = real(1.0) / kSrbMass;        // RN(1 / c): compile-time IEEE division
constexpr real kSrbInertiaRcp = real(1.0) / kSrbInertia;

MHPC_HD void srb_dynamics(const real* x, const real* u, const real* p, const real* s,
                          real* xd) {
  MHPC_NO_FMA
  xd[0] = x[3];
  xd[1] = x[4];
  xd[2] = x[5];
  xd[3] = div_const(s[0] * u[0], kSrbMass, kSrbMassRcp) + div_const(s[1] * u[2], kSrbMass, kSrbMassRcp);
  xd[4] = (div_const(s[0] * u[1], kSrbMass, kSrbMassRcp) + div_const(s[1] * u[3], kSrbMass, kSrbMassRcp)) +
          (-real(9.8100000000000005));
  const real tf = div_const((p[1] - x[1]) * u[0] - (p[0] - x[0]) * u[1], kSrbInertia, kSrbInertiaRcp);
  const real tb = div_const((p[3] - x[1]) * u[2] - (p[2] - x[0]) * u[3], kSrbInertia, kSrbInertiaRcp);
  xd[5] = s[0] * tf + s[1] * tb;
}

// Continuous Jacobians, dense row-major Ac (6x6) and Bc (6x4) (FBDynamics_par.c).
MHPC_HD void srb_jacobians(const real* x, const real* u, const real* p, const real* s,
                           real* Ac, real* Bc) {
  MHPC_NO_FMA
  for (int i = 0; i < 36; ++i) Ac[i] = real(0.0);
  for (int i = 0; i < 24; ++i) Bc[i] = real(0.0);
  Ac[5 * 6 + 0] = s[0] * (kSrbInvInertia * u[1]) + s[1] * (kSrbInvInertia * u[3]);
  Ac[5 * 6 + 1] = -(s[0] * (kSrbInvInertia * u[0]) + s[1] * (kSrbInvInertia * u[2]));
  Ac[0 * 6 + 3] = real(1.0);
  Ac[1 * 6 + 4] = real(1.0);
  Ac[2 * 6 + 5] = real(1.0);
  Bc[3 * 4 + 0] = kSrbInvMass * s[0];
  Bc[5 * 4 + 0] = s[0] * (kSrbInvInertia * (p[1] - x[1]));
  Bc[4 * 4 + 1] = kSrbInvMass * s[0];
  Bc[5 * 4 + 1] = -(s[0] * (kSrbInvInertia * (p[0] - x[0])));
  Bc[3 * 4 + 2] = kSrbInvMass * s[1];
  Bc[5 * 4 + 2] = s[1] * (kSrbInvInertia * (p[3] - x[1]));
  Bc[4 * 4 + 3] = kSrbInvMass * s[1];
  Bc[5 * 4 + 3] = -(s[1] * (kSrbInvInertia * (p[2] - x[0])));
}

}  // namespace MHPC_NS
