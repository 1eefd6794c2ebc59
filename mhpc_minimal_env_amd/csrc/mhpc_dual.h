// Forward-mode dual numbers for the Jacobian pass.
//
// The reference obtains every dynamics Jacobian from CasADi-generated straight-line C
// (Dyn_{FL,BS,FS}_par.c, Imp_{F,B}_par.c).  Here each lane of the
// partials kernel evaluates the hand-written model once in dual arithmetic along one
// tangent direction (one column of [A B] / Px), so a (knot, direction) grid gives every
// column in parallel with no generated code and exact (rounding-level) derivatives.
#pragma once
#include <math.h>

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

namespace mhpc {

struct Dual {
  double v;  // primal value
  double d;  // directional derivative
  MHPC_HD Dual() : v(0.0), d(0.0) {}
  MHPC_HD Dual(double a) : v(a), d(0.0) {}
  MHPC_HD Dual(double a, double b) : v(a), d(b) {}
};

MHPC_HD Dual operator+(Dual a, Dual b) { return Dual(a.v + b.v, a.d + b.d); }
MHPC_HD Dual operator-(Dual a, Dual b) { return Dual(a.v - b.v, a.d - b.d); }
MHPC_HD Dual operator-(Dual a) { return Dual(-a.v, -a.d); }
MHPC_HD Dual operator*(Dual a, Dual b) { return Dual(a.v * b.v, a.d * b.v + a.v * b.d); }
MHPC_HD Dual operator/(Dual a, Dual b) {
  const double q = a.v / b.v;
  return Dual(q, (a.d - q * b.d) / b.v);
}
MHPC_HD Dual operator+(Dual a, double b) { return Dual(a.v + b, a.d); }
MHPC_HD Dual operator+(double a, Dual b) { return Dual(a + b.v, b.d); }
MHPC_HD Dual operator-(Dual a, double b) { return Dual(a.v - b, a.d); }
MHPC_HD Dual operator-(double a, Dual b) { return Dual(a - b.v, -b.d); }
MHPC_HD Dual operator*(Dual a, double b) { return Dual(a.v * b, a.d * b); }
MHPC_HD Dual operator*(double a, Dual b) { return Dual(a * b.v, a * b.d); }
MHPC_HD Dual operator/(Dual a, double b) { return Dual(a.v / b, a.d / b); }
MHPC_HD Dual& operator+=(Dual& a, Dual b) { a = a + b; return a; }
MHPC_HD Dual& operator-=(Dual& a, Dual b) { a = a - b; return a; }
MHPC_HD Dual& operator*=(Dual& a, Dual b) { a = a * b; return a; }

// Scalar-generic elementary functions (double and Dual share the model source).
MHPC_HD double val(double a) { return a; }
MHPC_HD double val(Dual a) { return a.v; }

MHPC_HD void sin_cos(double a, double* s, double* c) {
#if defined(__HIP_DEVICE_COMPILE__)
  sincos(a, s, c);  // one shared argument reduction on the device
#else
  *s = sin(a);
  *c = cos(a);
#endif
}
MHPC_HD void sin_cos(Dual a, Dual* s, Dual* c) {
  double sv, cv;
  sin_cos(a.v, &sv, &cv);
  *s = Dual(sv, cv * a.d);
  *c = Dual(cv, -sv * a.d);
}
MHPC_HD double sqrt_(double a) { return sqrt(a); }
MHPC_HD Dual sqrt_(Dual a) {
  const double r = sqrt(a.v);
  return Dual(r, a.d / (2.0 * r));
}

}  // namespace mhpc
