// Whole-body dynamics evaluated by a lane pair: the line search's latency-bound dynamics
// wave gives each candidate two adjacent lanes (even lane: front leg, odd lane: back leg).
//
// The planar model is a tree: the two legs only meet in the base block of M, the base rows
// of the bias h, the Schur complement of the arrowhead factorisation (mhpc_model.h) and the
// contact KKT sums.  Each lane evaluates its own leg (two of the five link angles' sines /
// cosines, the two bodies' Jacobian products, the 2x2 leg block, its solve) and the pair
// swaps the per-leg terms of those shared quantities with one DPP move per word; both lanes
// then sum them in the order of the single-lane model (front thigh, front shank, back thigh,
// back shank; front leg before back leg), so every result -- and the base state both lanes
// carry -- is the single-lane model's value, bit for bit: neither model contracts a
// product into a sum (MHPC_NO_FMA, see mhpc_model.h), so equal operation order means equal
// rounding (tests/test_pair_host.py emulates the pair on the host with two threads;
// tests/test_gpu_kernels.py::test_wb_dynamics_pair_bitwise checks the device code).
// About 40 % fewer instructions per lane than one lane evaluating the whole model.
#pragma once
#include "mhpc_model.h"

namespace MHPC_NS {

// value held by the partner lane (lane ^ 1): DPP quad_perm [1, 0, 3, 2] (device only; the
// host pass of the kernels' translation unit only parses it)
MHPC_HD double pair_swap(double v) {
#if defined(__HIP_DEVICE_COMPILE__)
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  // mov_dpp: no "old" operand to materialise (every lane has a valid source in a quad_perm)
  const unsigned lo = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)b, 0xB1, 0xF, 0xF, false);
  const unsigned hi = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)(b >> 32), 0xB1, 0xF, 0xF, false);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
#elif defined(MHPC_PAIR_HOST_SWAP)
  return mhpc_host_pair_swap(v);  // test-only host emulation of the lane pair (two threads)
#else
  return v;
#endif
}
MHPC_HD float pair_swap(float v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
#elif defined(MHPC_PAIR_HOST_SWAP)
  return (float)mhpc_host_pair_swap((double)v);
#else
  return v;
#endif
}

// value held by the pair's even (E = 0) / odd (E = 1) lane, on both lanes: DPP quad_perm
// [0, 0, 2, 2] / [1, 1, 3, 3] -- a broadcast inside the pair, no lane-dependent select
template <int E>
MHPC_HD double pair_from(double v) {
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr int ctl = E ? 0xF5 : 0xA0;
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)b, ctl, 0xF, 0xF, false);
  const unsigned hi = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)(b >> 32), ctl, 0xF, 0xF, false);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
#else
  return v;  // (host: only the lane-parity forms below are used)
#endif
}
template <int E>
MHPC_HD float pair_from(float v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), E ? 0xF5 : 0xA0, 0xF, 0xF, false));
#else
  return v;
#endif
}
// The stance lane's value (odd lane when sback) on both lanes; `mine` = this lane is it.
template <bool SBACK>
MHPC_HD real pair_stance(bool mine, real v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return pair_from<SBACK ? 1 : 0>(v);
#else
  const real o = pair_swap(v);
  return mine ? v : o;
#endif
}

// Jacobian of a point of the own leg (leg_point_jac with the hip side as data: sg = +1
// front, -1 back), same expressions.
MHPC_HD void pair_point_jac(const LegGeo<real, real>& L, real sg, real sth,
                                               real cth, real l1, real l2, real jx[5], real jz[5],
                                               real* jdx, real* jdz) {
  MHPC_NO_FMA_WB
  const real tx1 = -l1 * L.c1, tz1 = l1 * L.s1;
  const real tx2 = -l2 * L.c2, tz2 = l2 * L.s2;
  jx[0] = real(1.0); jz[0] = real(0.0);
  jx[1] = real(0.0); jz[1] = real(1.0);
  jx[4] = tx2;    jz[4] = tz2;
  jx[3] = tx1 + tx2;
  jz[3] = tz1 + tz2;
  jx[2] = mad(-sg * kHipX, sth, jx[3]);
  jz[2] = mad(-sg * kHipX, cth, jz[3]);
  *jdx = mad(L.w1 * L.w1, l1 * L.s1, L.w2 * L.w2 * (l2 * L.s2));
  *jdz = mad(L.w1 * L.w1, l1 * L.c1, L.w2 * L.w2 * (l2 * L.c2));
}

// Own-leg part of M and h (add_leg): the base entries per body (M(2,0), M(2,1), M(2,2),
// h0, h1, h2 of thigh / shank, summed by the caller in model order) and the leg's own
// entries (local index 3 = hip, 4 = knee; the coupling rows and the 2x2 block, h of the
// leg joints), accumulated from zero as add_leg does.
struct PairLegMH {
  real base[2][6];  // [body][M20, M21, M22, h0, h1, h2]
  real Mh[3], Mk[3];   // coupling: M(hip, 0..2), M(knee, 0..2)
  real Mhh, Mkh, Mkk;  // leg block
  real hh, hk;         // h of the hip / knee joint
};
MHPC_HD void pair_leg_mass_bias(const LegGeo<real, real>& L, real sg, real sth,
                                                   real cth, real thd, PairLegMH& o) {
  MHPC_NO_FMA_WB  // as add_leg (mhpc_model.h): the per-body terms are rounded before any sum
  const real thd2 = thd * thd;
  const real hax = (-sg * kHipX) * cth * thd2;
  const real haz = (sg * kHipX) * sth * thd2;
  real Ml[5][5];  // local lower triangle rows 3, 4 (cols 0..4) -- rows 0..2 go to base[]
#pragma unroll
  for (int a = 3; a < 5; ++a)
#pragma unroll
    for (int c = 0; c < 5; ++c) Ml[a][c] = real(0.0);
  real hl[5] = {real(0.0), real(0.0), real(0.0), real(0.0), real(0.0)};
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    real jx[5], jz[5], jdx, jdz, m, ic;
    if (b == 0) {
      pair_point_jac(L, sg, sth, cth, kThighCom, real(0.0), jx, jz, &jdx, &jdz);
      m = kThighMass; ic = kThighInertiaCom;
    } else {
      pair_point_jac(L, sg, sth, cth, kThighLen, kShankCom, jx, jz, &jdx, &jdz);
      m = kShankMass; ic = kShankInertiaCom;
    }
    const int nc = b == 0 ? 4 : 5;
    jdx += hax;
    jdz += haz;
    const real ax = jdx, az = jdz + kGrav;
    real* bb = o.base[b];
#pragma unroll
    for (int a = 0; a < 5; ++a) {
      if (a >= nc) continue;
      const real dh = m * mad(jx[a], ax, jz[a] * az);
      if (a < 3) bb[3 + a] = dh;
      else hl[a] += dh;
#pragma unroll
      for (int c = 0; c <= a; ++c) {
        if (a < 2 && c < 2) continue;  // constant entries (the body masses), summed by the caller
        real v = m * mad(jx[a], jx[c], jz[a] * jz[c]);
        if (a >= 2 && c >= 2) v += ic;
        if (a == 2) bb[c] = v;  // M(2, c), c = 0, 1, 2
        else Ml[a][c] += v;
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) { o.Mh[c] = Ml[3][c]; o.Mk[c] = Ml[4][c]; }
  o.Mhh = Ml[3][3];
  o.Mkh = Ml[4][3];
  o.Mkk = Ml[4][4];
  o.hh = hl[3];
  o.hk = hl[4];
}

// Order the own / partner value of a per-leg quantity as (front, back): the even (front)
// lane's and the odd (back) lane's value, broadcast inside the pair.
MHPC_HD void pair_order(bool back, real own, real* fr, real* bk) {
#if defined(__HIP_DEVICE_COMPILE__)
  (void)back;
  *fr = pair_from<0>(own);
  *bk = pair_from<1>(own);
#else
  const real oth = pair_swap(own);
  *fr = back ? oth : own;
  *bk = back ? own : oth;
#endif
}

// front + back of a per-leg quantity, the same on both lanes without ordering them: a sum
// of two terms does not depend on their order (the single-lane model sums front + back).
MHPC_HD real pair_sum(real own) {
  MHPC_NO_FMA_WB
  return own + pair_swap(own);
}

// Arrowhead solve of the pair: rhs = (base part rb[3] identical on both lanes, own-leg
// part rl[2]); returns the base result xb[3] (identical on both lanes) and the own-leg
// result xl[2].  Same operations and order as arrow_solve.
struct PairFactor {
  real Li[3];      // own leg block inverse (a, b, c of [[a b][b c]]^-1)
  real Z[2][3];    // own leg Z = Ml^-1 M_lb
  real Si[6];      // inverse base Schur complement (identical on both lanes)
  real Mh[3], Mk[3];  // own coupling rows (M(i0, j), M(i1, j))
};
MHPC_HD void pair_solve(const PairFactor& F, bool back, const real rb[3],
                                           const real rl[2], real xb[3], real xl[2]) {
  MHPC_NO_FMA_WB
  const real w0 = mad(F.Li[0], rl[0], F.Li[1] * rl[1]);
  const real w1 = mad(F.Li[1], rl[0], F.Li[2] * rl[1]);
  const real t0 = mad(F.Mh[0], w0, F.Mk[0] * w1);
  const real t1 = mad(F.Mh[1], w0, F.Mk[1] * w1);
  const real t2 = mad(F.Mh[2], w0, F.Mk[2] * w1);
  // base rows minus front + back (arrow_solve)
  const real r0 = rb[0] - pair_sum(t0), r1 = rb[1] - pair_sum(t1), r2 = rb[2] - pair_sum(t2);
  const real x0 = mad(F.Si[3], r2, mad(F.Si[1], r1, F.Si[0] * r0));
  const real x1 = mad(F.Si[4], r2, mad(F.Si[2], r1, F.Si[1] * r0));
  const real x2 = mad(F.Si[5], r2, mad(F.Si[4], r1, F.Si[3] * r0));
  xb[0] = x0; xb[1] = x1; xb[2] = x2;
  xl[0] = w0 - mad(F.Z[0][2], x2, mad(F.Z[0][1], x1, F.Z[0][0] * x0));
  xl[1] = w1 - mad(F.Z[1][2], x2, mad(F.Z[1][1], x1, F.Z[1][0] * x0));
}

// What the pair dynamics needs of the state alone (geometry, mass matrix factor, bias): it
// does not depend on the controls, so the line search evaluates it while the knot's feedback
// operands are still on their way from LDS (wb_pair_prep, then the feedback, then
// wb_pair_finish -- the same operations as wb_dynamics_pair, in the same order per value).
struct WbPairPrep {
  LegGeo<real, real> L;
  real sg, sth, cth;
  real hh, hk;     // own leg joint bias
  real hb[3];      // base bias
  PairFactor F;
};
MHPC_HD void wb_pair_prep(const real* x, bool back, WbPairPrep& P, const SinCosK& K = kSinCosK) {
  MHPC_NO_FMA_WB
  const real sg = back ? -real(1.0) : real(1.0);
  // geometry: the body pitch and the own leg's two links
  const real qh = back ? x[5] : x[3], qk = back ? x[6] : x[4];
  const real qhd = back ? x[12] : x[10], qkd = back ? x[13] : x[11];
  LegGeo<real, real>& L = P.L;
  const real a1 = x[2] + qh;
  const real a2 = a1 + qk;
  real sv[3], cv[3];
  sin_cos_n<3>({x[2], a1, a2}, sv, cv, K);
  const real sth = sv[0], cth = cv[0];
  L.s1 = sv[1]; L.c1 = cv[1];
  L.s2 = sv[2]; L.c2 = cv[2];
  L.w1 = x[9] + qhd;
  L.w2 = L.w1 + qkd;
  P.sg = sg; P.sth = sth; P.cth = cth;
  PairLegMH lm;
  pair_leg_mass_bias(L, sg, sth, cth, x[9], lm);
  // base block and base bias: body constant + (front leg + back leg), each leg thigh +
  // shank (wb_mass_bias + add_leg order)
  real bs[6];  // M20, M21, M22, h0, h1, h2
  const real init[6] = {real(0.0), real(0.0), kBodyInertia, real(0.0), kBodyMass * kGrav,
                        real(0.0)};
#pragma unroll
  for (int e = 0; e < 6; ++e) bs[e] = init[e] + pair_sum(lm.base[0][e] + lm.base[1][e]);
  // M00 = M11 = body + leg masses (constant), M10 = 0
  real M00 = kBodyMass, M11 = kBodyMass;
  M00 += kThighMass; M11 += kThighMass;
  M00 += kShankMass; M11 += kShankMass;
  M00 += kThighMass; M11 += kThighMass;
  M00 += kShankMass; M11 += kShankMass;
  const real M10 = real(0.0), M20 = bs[0], M21 = bs[1], M22 = bs[2];
  // arrowhead factorisation (arrow_factor), own leg block, Schur terms swapped
  PairFactor& F = P.F;
  {
    const real a = lm.Mhh, b = lm.Mkh, c = lm.Mkk;
    const real rdet = pivot_rcp(mad(a, c, -(b * b)));
    F.Li[0] = c * rdet;
    F.Li[1] = -b * rdet;
    F.Li[2] = a * rdet;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const real m0 = lm.Mh[j], m1 = lm.Mk[j];
      F.Z[0][j] = mad(F.Li[0], m0, F.Li[1] * m1);
      F.Z[1][j] = mad(F.Li[1], m0, F.Li[2] * m1);
      F.Mh[j] = m0;
      F.Mk[j] = m1;
    }
  }
  const real* z0 = F.Z[0];
  const real* z1 = F.Z[1];
  const real t[6] = {mad(lm.Mh[0], z0[0], lm.Mk[0] * z1[0]), mad(lm.Mh[1], z0[0], lm.Mk[1] * z1[0]),
                     mad(lm.Mh[1], z0[1], lm.Mk[1] * z1[1]), mad(lm.Mh[2], z0[0], lm.Mk[2] * z1[0]),
                     mad(lm.Mh[2], z0[1], lm.Mk[2] * z1[1]), mad(lm.Mh[2], z0[2], lm.Mk[2] * z1[2])};
  real s[6] = {M00, M10, M11, M20, M21, M22};  // s00, s10, s11, s20, s21, s22
#pragma unroll
  for (int e = 0; e < 6; ++e) s[e] -= pair_sum(t[e]);  // minus front + back (arrow_factor)
  {
    const real s00 = s[0], s10 = s[1], s11 = s[2], s20 = s[3], s21 = s[4], s22 = s[5];
    const real c00 = mad(s11, s22, -(s21 * s21));
    const real c10 = mad(s21, s20, -(s10 * s22));
    const real c20 = mad(s10, s21, -(s11 * s20));
    const real rdet = pivot_rcp(mad(s20, c20, mad(s10, c10, s00 * c00)));
    F.Si[0] = c00 * rdet;
    F.Si[1] = c10 * rdet;
    F.Si[2] = mad(s00, s22, -(s20 * s20)) * rdet;
    F.Si[3] = c20 * rdet;
    F.Si[4] = mad(s20, s10, -(s00 * s21)) * rdet;
    F.Si[5] = mad(s00, s11, -(s10 * s10)) * rdet;
  }
  P.hh = lm.hh;
  P.hk = lm.hk;
  P.hb[0] = bs[3]; P.hb[1] = bs[4]; P.hb[2] = bs[5];
}

template <bool SBACK>
MHPC_HD void wb_stance_pair(const real* x, const LegGeo<real, real>& L, real sg, real sth,
                            real cth, bool back, const PairFactor& F, real v[7], real* y);

// The controls' part: M v = S'u - h, the contact correction, xdot.
MHPC_HD void wb_pair_finish(const real* x, const real u_own[2], int mode, bool back,
                            const WbPairPrep& P, real* xdot, real* y) {
  MHPC_NO_FMA_WB
  // unconstrained accelerations: M v = S'u - h
  real vb[3], vl[2];
  {
    const real rb[3] = {-P.hb[0], -P.hb[1], -P.hb[2]};
    const real rl[2] = {u_own[0] - P.hh, u_own[1] - P.hk};
    pair_solve(P.F, back, rb, rl, vb, vl);
  }
  // full v in model order (front leg, back leg)
  real v[7];
  v[0] = vb[0]; v[1] = vb[1]; v[2] = vb[2];
  pair_order(back, vl[0], &v[3], &v[5]);
  pair_order(back, vl[1], &v[4], &v[6]);
#pragma unroll
  for (int i = 0; i < 4; ++i) y[i] = real(0.0);
  if (mode == 1) wb_stance_pair<true>(x, P.L, P.sg, P.sth, P.cth, back, P.F, v, y);
  else if (mode == 3) wb_stance_pair<false>(x, P.L, P.sg, P.sth, P.cth, back, P.F, v, y);
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    xdot[i] = x[7 + i];
    xdot[7 + i] = v[i];
  }
}

// x (14, identical on both lanes of the pair), u_own = the own leg's two joint torques.
// Returns xdot (14) and y (4), identical on both lanes.  mode as wb_dynamics.
MHPC_HD void wb_dynamics_pair(const real* x, const real u_own[2], int mode,
                                                 bool back, real* xdot, real* y) {
  WbPairPrep P;
  wb_pair_prep(x, back, P);
  wb_pair_finish(x, u_own, mode, back, P, xdot, y);
}

// The contact KKT correction of a stance mode (kkt_contact), SBACK = the back foot is down
// (mode 1; the front foot: mode 3): the stance foot's lane evaluates the foot Jacobian and
// J-dot qdot (wb_foot_jac_full), broadcast to the partner.
template <bool SBACK>
MHPC_HD void wb_stance_pair(const real* x, const LegGeo<real, real>& L, real sg, real sth,
                            real cth, bool back, const PairFactor& F, real v[7], real* y) {
  MHPC_NO_FMA_WB
  {
    const bool sback = SBACK;
    const bool mine = sback == back;
    real jx[5], jz[5], jdx, jdz;
    pair_point_jac(L, sg, sth, cth, kThighLen, kShankLen, jx, jz, &jdx, &jdz);
    const real thd2 = x[9] * x[9];
    real jd0 = jdx + (-sg * kHipX) * cth * thd2;
    real jd1 = jdz + (sg * kHipX) * sth * thd2;
    // the stance lane's values on both lanes
    real Jb[2][3], Jl[2][2];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      Jb[0][a] = pair_stance<SBACK>(mine, jx[a]);
      Jb[1][a] = pair_stance<SBACK>(mine, jz[a]);
    }
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      Jl[0][a] = pair_stance<SBACK>(mine, jx[3 + a]);
      Jl[1][a] = pair_stance<SBACK>(mine, jz[3 + a]);
    }
    jd0 = pair_stance<SBACK>(mine, jd0);
    jd1 = pair_stance<SBACK>(mine, jd1);
    // full J rows in model order (zeros on the swing leg's columns)
    real J[2][7];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
#pragma unroll
      for (int i = 0; i < 7; ++i) J[r][i] = real(0.0);
#pragma unroll
      for (int a = 0; a < 3; ++a) J[r][a] = Jb[r][a];
      J[r][sback ? 5 : 3] = Jl[r][0];
      J[r][sback ? 6 : 4] = Jl[r][1];
    }
    // Y = M^-1 J' (kkt_contact), own-leg rhs = the stance leg's J entries or zero
    real Y[2][7];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const real rb[3] = {Jb[r][0], Jb[r][1], Jb[r][2]};
      const real rl[2] = {mine ? Jl[r][0] : real(0.0), mine ? Jl[r][1] : real(0.0)};
      real yb[3], yl[2];
      pair_solve(F, back, rb, rl, yb, yl);
      Y[r][0] = yb[0]; Y[r][1] = yb[1]; Y[r][2] = yb[2];
      pair_order(back, yl[0], &Y[r][3], &Y[r][5]);
      pair_order(back, yl[1], &Y[r][4], &Y[r][6]);
    }
    real A00 = real(0.0), A01 = real(0.0), A11 = real(0.0);
    real r0 = -jd0, r1 = -jd1;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      A00 = mad(J[0][i], Y[0][i], A00);
      A01 = mad(J[0][i], Y[1][i], A01);
      A11 = mad(J[1][i], Y[1][i], A11);
      r0 = mad(-J[0][i], v[i], r0);
      r1 = mad(-J[1][i], v[i], r1);
    }
    const real rdet = pivot_rcp(mad(A00, A11, -(A01 * A01)));
    const real lam0 = mad(A11, r0, -(A01 * r1)) * rdet;
    const real lam1 = mad(A00, r1, -(A01 * r0)) * rdet;
#pragma unroll
    for (int i = 0; i < 7; ++i) v[i] += mad(Y[0][i], lam0, Y[1][i] * lam1);
    y[sback ? 2 : 0] = lam0;
    y[sback ? 3 : 1] = lam1;
  }
}

}  // namespace MHPC_NS
