// Forward-mode dual numbers for the Jacobian pass.
//
// The reference obtains every dynamics Jacobian from CasADi-generated straight-line C
// (Dyn_{FL,BS,FS}_par.c, Imp_{F,B}_par.c).  Here each lane of the
// partials kernel evaluates the hand-written model once in dual arithmetic along one
// tangent direction (one column of [A B] / Px), so a (knot, direction) grid gives every
// column in parallel with no generated code and exact (rounding-level) derivatives.
#pragma once
#include <math.h>

#include "mhpc_real.h"

#if defined(__HIPCC__)
#define MHPC_HD __host__ __device__ __forceinline__
#else
#define MHPC_HD inline
#endif

// Unfused multiply-add inside a block: the SRB kernels keep FBDynamics.c's rounding exactly.
#if defined(__clang__)
#define MHPC_NO_FMA _Pragma("clang fp contract(off)")
#else
#define MHPC_NO_FMA
#endif

// fp32 build only: no contraction in the line search and the cost functions.  In fp32 the
// SLP vectorizer packs scalar operations into v_pk_* pairs differently in each line-search
// variant, and a packed multiply loses the contract flag of a scalar one, so the same
// expression would fuse in one variant and not in another; with no contraction the rounding
// is the same whatever is packed (tests/test_gpu_variants.py, fp32).  fp64 has no packed
// arithmetic on gfx950, so its contraction is the same in every variant.
#if defined(__clang__) && defined(MHPC_FP32)
#define MHPC_NO_FMA_F32 _Pragma("clang fp contract(off)")
#else
#define MHPC_NO_FMA_F32
#endif
// Costs and their sums, in both precisions: a cost evaluation is inlined into the loops of
// several kernels (line search, forward_sweep(0), trial rollouts) and its last product could
// otherwise fuse with the caller's accumulation in one of them and not in another.
#if defined(__clang__)
#define MHPC_NO_FMA_COST _Pragma("clang fp contract(off)")
#else
#define MHPC_NO_FMA_COST
#endif

namespace MHPC_NS {

struct Dual {
  real v;  // primal value
  real d;  // directional derivative
  MHPC_HD Dual() : v(real(0.0)), d(real(0.0)) {}
  MHPC_HD Dual(real a) : v(a), d(real(0.0)) {}
  MHPC_HD Dual(real a, real b) : v(a), d(b) {}
};

MHPC_HD Dual operator+(Dual a, Dual b) { return Dual(a.v + b.v, a.d + b.d); }
MHPC_HD Dual operator-(Dual a, Dual b) { return Dual(a.v - b.v, a.d - b.d); }
MHPC_HD Dual operator-(Dual a) { return Dual(-a.v, -a.d); }
MHPC_HD Dual operator*(Dual a, Dual b) { return Dual(a.v * b.v, a.d * b.v + a.v * b.d); }
MHPC_HD Dual operator/(Dual a, Dual b) {
  const real q = a.v / b.v;
  return Dual(q, (a.d - q * b.d) / b.v);
}
MHPC_HD Dual operator+(Dual a, real b) { return Dual(a.v + b, a.d); }
MHPC_HD Dual operator+(real a, Dual b) { return Dual(a + b.v, b.d); }
MHPC_HD Dual operator-(Dual a, real b) { return Dual(a.v - b, a.d); }
MHPC_HD Dual operator-(real a, Dual b) { return Dual(a - b.v, -b.d); }
MHPC_HD Dual operator*(Dual a, real b) { return Dual(a.v * b, a.d * b); }
MHPC_HD Dual operator*(real a, Dual b) { return Dual(a * b.v, a * b.d); }
MHPC_HD Dual operator/(Dual a, real b) { return Dual(a.v / b, a.d / b); }
MHPC_HD Dual& operator+=(Dual& a, Dual b) { a = a + b; return a; }
MHPC_HD Dual& operator-=(Dual& a, Dual b) { a = a - b; return a; }
MHPC_HD Dual& operator*=(Dual& a, Dual b) { a = a * b; return a; }

// Fused a * b + c, written out where the whole-body models want it: the models are compiled
// without contraction (MHPC_NO_FMA_WB, so that the line search's lane pair and the single
// lane round alike), and every fused product is spelled the same way in both.  Dual: the
// primal fused, the tangent (a b)' + c' (the partials compare to the reference at 1e-9).
MHPC_HD real mad(real a, real b, real c) { return fma(a, b, c); }
MHPC_HD Dual mad(Dual a, Dual b, Dual c) { return Dual(fma(a.v, b.v, c.v), fma(a.d, b.v, fma(a.v, b.d, c.d))); }
MHPC_HD Dual mad(real a, Dual b, Dual c) { return Dual(fma(a, b.v, c.v), fma(a, b.d, c.d)); }
MHPC_HD Dual mad(Dual a, real b, Dual c) { return Dual(fma(a.v, b, c.v), fma(a.d, b, c.d)); }
MHPC_HD Dual mad(Dual a, Dual b, real c) { return Dual(fma(a.v, b.v, c), fma(a.d, b.v, a.v * b.d)); }
MHPC_HD Dual mad(real a, real b, Dual c) { return Dual(fma(a, b, c.v), c.d); }
MHPC_HD Dual mad(real a, Dual b, real c) { return Dual(fma(a, b.v, c), a * b.d); }
MHPC_HD Dual mad(Dual a, real b, real c) { return Dual(fma(a.v, b, c), a.d * b); }

// 1 / a of a whole-body model pivot (the 2x2 leg blocks, the 3x3 base Schur complement, the
// 2x2 contact KKT block).  fp64 device code: the hardware reciprocal estimate refined by two
// Newton steps (within an ulp of the IEEE quotient, about half the instructions and dependent
// steps of the division sequence on the serial knot chain), the estimate itself where the
// refinement is not finite (a = 0, +-inf, NaN: the IEEE value).  The fp32 build keeps the
// IEEE quotient: its C5 cost error is chaotic in the last bits of the model (one Newton step
// from the fp32 estimate moved the worst of 64 problems from 1.8e-3 to 6.0e-3, past the
// test's 5e-3 target).  The single-lane, lane-pair and dual-number models all take it, so they
// still agree bit for bit where they must (tests/test_pair_host.py, test_gpu_kernels.py).
MHPC_HD real pivot_rcp(real a) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(MHPC_FP32)
  const double r = __builtin_amdgcn_rcp(a);
  const double r1 = fma(r, fma(-a, r, 1.0), r);
  const double r2 = fma(r1, fma(-a, r1, 1.0), r1);
  return __builtin_isfinite(r2) ? r2 : r;
#else
  return real(1.0) / a;
#endif
}
MHPC_HD Dual pivot_rcp(Dual a) {
#ifdef MHPC_FP32
  return Dual(real(1.0), real(0.0)) / a;
#else
  const real r = pivot_rcp(a.v);
  return Dual(r, -(a.d * r) * r);
#endif
}

// Scalar-generic elementary functions (real and Dual share the model source).
MHPC_HD real val(real a) { return a; }
MHPC_HD real val(Dual a) { return a.v; }
MHPC_HD real tangent(real) { return real(0.0); }
MHPC_HD real tangent(Dual a) { return a.d; }

// The short sin / cos reduction's and kernels' constants (below).  A caller may pass a copy
// held in VGPRs (a knot loop: no per-knot s_mov pairs materialising them, gfx950 has no
// 64-bit literal operand); the values, hence the results, are the same.
struct SinCosK {
  double c[15];
};
constexpr SinCosK kSinCosK = {{0.63661977236758138,  // 2 / pi
                               1.5707963267948966,   // pi/2, high part
                               6.123233995736766e-17,  // pi/2 - high part
                               8.33333333332248946124e-03, -1.98412698298579493134e-04,
                               2.75573137070700676789e-06, -2.50507602534068634195e-08,
                               1.58969099521155010221e-10, -1.66666666666666324348e-01,
                               4.16666666666666019037e-02, -1.38888888888741095749e-03,
                               2.48015872894767294178e-05, -2.75573143513906633035e-07,
                               2.08757232129817482790e-09, -1.13596475577881948265e-11}};

#ifndef MHPC_FP32
// sin and cos of a link angle: one Cody-Waite reduction by pi/2 (two-part pi/2, FMA) and
// the fdlibm kernels on |r| <= pi/4 (< 0.75 ulp each); <= 1.5 ulp overall, checked against
// long double on |a| <= 60.  About half the instructions of the library sincos, whose
// reduction carries a double-double and a Payne-Hanek path for huge arguments -- kept here
// only for |a| > 1e5 (a diverged rollout), where the short reduction loses accuracy.
MHPC_HD void sin_cos_short(double a, double* s, double* c, const SinCosK& K = kSinCosK) {
  const double k = rint(a * K.c[0]);
  double r = fma(-k, K.c[1], a);
  r = fma(-k, K.c[2], r);
  const double z = r * r;
  const double ps = K.c[3] + z * (K.c[4] + z * (K.c[5] + z * (K.c[6] + z * K.c[7])));
  const double sn = r + (z * r) * (K.c[8] + z * ps);
  const double pc = z * (K.c[9] + z * (K.c[10] + z * (K.c[11] + z * (K.c[12] + z * (K.c[13] + z * K.c[14])))));
  const double hz = 0.5 * z, w = 1.0 - hz;
  const double cs = w + (((1.0 - w) - hz) + z * pc);
  const int n = (int)k & 3;
  const double so = (n & 1) ? cs : sn, co = (n & 1) ? sn : cs;
  *s = (n & 2) ? -so : so;
  *c = ((n + 1) & 2) ? -co : co;
}
#endif

MHPC_HD void sin_cos(real a, real* s, real* c) {
#ifdef MHPC_FP32
#if defined(__HIP_DEVICE_COMPILE__)
  sincosf(a, s, c);
#else
  *s = sinf(a);
  *c = cosf(a);
#endif
#elif defined(__HIP_DEVICE_COMPILE__)
  // the library path as a wave-uniform branch (taken only when some lane's argument is out
  // of the short reduction's range): no exec-mask join in the knot loops
  sin_cos_short(a, s, c);
  if (__builtin_amdgcn_ballot_w64(!(fabs(a) <= 1e5))) {
    real sl, cl;
    sincos(a, &sl, &cl);
    const bool big = !(fabs(a) <= 1e5);
    *s = big ? sl : *s;
    *c = big ? cl : *c;
  }
#else
  if (fabs(a) <= 1e5) {
    sin_cos_short(a, s, c);
  } else {
#if defined(__HIP_DEVICE_COMPILE__)
    sincos(a, s, c);
#else
    *s = sin(a);
    *c = cos(a);
#endif
  }
#endif
}
// sin_cos of N angles at once: the short reductions and polynomials of all N side by side
// (one set of constants, interleaved chains) and one wave-uniform library fallback for them
// all; per angle the same value as sin_cos.
template <int N>
MHPC_HD void sin_cos_n(const real (&a)[N], real (&s)[N], real (&c)[N], const SinCosK& K = kSinCosK) {
#if !defined(MHPC_FP32) && defined(__HIP_DEVICE_COMPILE__)
  bool big = false;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    sin_cos_short(a[i], &s[i], &c[i], K);
    big = big || !(fabs(a[i]) <= 1e5);
  }
  if (__builtin_amdgcn_ballot_w64(big)) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      real sl, cl;
      sincos(a[i], &sl, &cl);
      const bool bi = !(fabs(a[i]) <= 1e5);
      s[i] = bi ? sl : s[i];
      c[i] = bi ? cl : c[i];
    }
  }
#else
  (void)K;
#pragma unroll
  for (int i = 0; i < N; ++i) sin_cos(a[i], &s[i], &c[i]);
#endif
}
MHPC_HD void sin_cos(Dual a, Dual* s, Dual* c) {
  real sv, cv;
  sin_cos(a.v, &sv, &cv);
  *s = Dual(sv, cv * a.d);
  *c = Dual(cv, -sv * a.d);
}
MHPC_HD real sqrt_(real a) { return sqrt(a); }
MHPC_HD Dual sqrt_(Dual a) {
  const real r = sqrt(a.v);
  return Dual(r, a.d / (real(2.0) * r));
}

}  // namespace MHPC_NS
