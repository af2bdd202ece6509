// sk_trig.hpp — branch-free fp64 sin+cos for the fused step kernels
// (host- and device-compilable so tests can check it against glibc on CPU).
//
// Why: ocml's sincos splits the basic block on its large-argument test, so
// the four independent sincos of a tick (two player moves, two projectiles)
// ran as four serial dependency chains at one wave per SIMD.  This version has
// no branches for |x| < 2^20*pi/2 (1.6e6 rad) and reports larger / non-finite
// arguments through `ok` so the caller can redo those lanes (rare, wave-
// uniform branch after all four are issued).
//
// Algorithm: Cody-Waite reduction by pi/2 split in four parts (the fdlibm /
// musl constants, public domain), every rounding error carried so the
// reduction is branch-free, then musl's degree-13/14 minimax kernels on
// [-pi/4, pi/4] with the reduced argument's tail, their polynomials evaluated
// with explicit fmas (0.1 us less per 65,536-game k_step than separate
// products, profiles/r02_step_ablation.jsonl).  Measured against glibc:
// |error| <= 1 ulp, exact at +-0 (sin = +-0, cos = 1) — the only argument
// where the game's int(round(x - sin(r)*3*s)) has exact ties.  Compile with
// -ffp-contract=off: the reduction relies on separately rounded products.
#pragma once
#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define SKT_HD __host__ __device__ __forceinline__
#else
#define SKT_HD static inline
#endif

namespace sktrig {

struct SinCos {
  double s, c;
};

// musl __sin(x, y, 1): sin(x + y) for |x| <= pi/4
SKT_HD double ksin(double x, double y) {
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  double z = x * x;
  double w = z * z;
#ifndef SK_TRIG_NOFMA  // explicit fmas in the polynomial (A/B: -DSK_TRIG_NOFMA)
  double r = fma(z * w, fma(z, S6, S5), fma(z, fma(z, S4, S3), S2));
  double v = z * x;
  return x - (fma(z, fma(-v, r, 0.5 * y), -y) - v * S1);
#else
  double r = S2 + z * (S3 + z * S4) + z * w * (S5 + z * S6);
  double v = z * x;
  return x - ((z * (0.5 * y - v * r) - y) - v * S1);
#endif
}

// musl __cos(x, y): cos(x + y) for |x| <= pi/4
SKT_HD double kcos(double x, double y) {
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  double z = x * x;
  double w = z * z;
#ifndef SK_TRIG_NOFMA
  double r = fma(z, fma(z, fma(z, C3, C2), C1), w * w * fma(z, fma(z, C6, C5), C4));
  double hz = 0.5 * z;
  w = 1.0 - hz;
  return w + (((1.0 - w) - hz) + fma(z, r, -x * y));
#else
  double r = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6));
  double hz = 0.5 * z;
  w = 1.0 - hz;
  return w + (((1.0 - w) - hz) + (z * r - x * y));
#endif
}

// sin and cos of x; ok = false for |x| >= 2^20*pi/2 or non-finite x (result
// then meaningless: recompute with the library routine)
SKT_HD SinCos sincos_bf(double x, bool* ok) {
#ifdef SK_ABL_NOTRIG  // timing ablation only: wrong values, same data flow
  *ok = fabs(x) < 1647099.3291652855;
  return SinCos{x * 0.125, 1.0 - x * 0.0625};
#endif
  const double invpio2 = 6.36619772367581382433e-01;
  const double pio2_1 = 1.57079632673412561417e+00;  // first 33 bits of pi/2
  const double pio2_2 = 6.07710050630396597660e-11;  // next 33 bits
  const double pio2_3 = 2.02226624871116645580e-21;  // next 33 bits
  const double pio2_3t = 8.47842766036889956997e-32; // pi/2 - (pio2_1 + pio2_2 + pio2_3)
  *ok = fabs(x) < 1647099.3291652855;  // false for NaN too
  double fn = rint(x * invpio2);
  // x - fn*pi/2 with pi/2 = pio2_1 + pio2_2 + pio2_3 + pio2_3t; each product
  // fn*pio2_k is exact (33-bit constants, |fn| < 2^20) and the rounding error
  // of every subtraction is carried (e2, e3), so no refinement branch is
  // needed (relative error of y0+y1 <= 4e-18 against a quad reference,
  // including arguments next to multiples of pi/2).
  double r = x - fn * pio2_1;
  double t = r;
  double w = fn * pio2_2;
  r = t - w;
  double e2 = (t - r) - w;
  t = r;
  w = fn * pio2_3;
  r = t - w;
  double e3 = (t - r) - w;
  w = fn * pio2_3t - e3 - e2;
  double y0 = r - w;
  double y1 = (r - y0) - w;
  double ks = ksin(y0, y1), kc = kcos(y0, y1);
  int n = (int)fn & 3;
  SinCos o;
  o.s = (n & 1) ? kc : ks;
  o.c = (n & 1) ? ks : kc;
  if (n == 1 || n == 2) o.c = -o.c;
  if (n >= 2) o.s = -o.s;
  o.s = (x == 0.0) ? x : o.s;  // sin(-0) = -0 like libm
  return o;
}

}  // namespace sktrig

namespace sktrig {

// ---------------------------------------------------------------- fast path
// The step only needs int(round(p - sin(r)*k)) for small k (3 or 5), so the
// sin/cos values themselves never reach the state: an fp32 sin/cos of the
// fp64-reduced argument decides the rounding whenever the fp32 delta is
// farther than its error bound from a half-integer; the rare lanes within
// the bound redo the move with the fp64 sincos_bf above (callers do that).
//
// Reduction: fn = rint(x*2/pi); y = (x - fn*pio2_1) - fn*pio2_2 in fp64 (both
// products exact for |fn| < 2^20; the dropped tail fn*(pi/2 - pio2_1 -
// pio2_2) is below 2.1e-21*2^20 = 2.2e-15).  Then y -> fp32 (|err| <= 4.7e-8
// on |y| <= pi/4) and the Cephes sinf/cosf minimax polynomials in fp32 FMAs.
// SKT_FAST_ERR bounds |sin_f - sin(x)| and |cos_f - cos(x)| for every x with
// ok = true; tests/trig_check.cpp measures the maximum against long-double
// sinl/cosl (about 1.3e-7) and checks it stays below half this bound.
#define SKT_FAST_ERR 3.0e-7f

struct SinCosF {
  float s, c;
};

// Cephes sinf / cosf minimax polynomials on [-pi/4, pi/4] (fp32 FMAs)
SKT_HD SinCosF sincos_poly(float yf) {
  const float z = yf * yf;
  const float ps = fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
  const float pc = fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f);
  SinCosF o;
  o.s = fmaf(yf * z, ps, yf);
  o.c = fmaf(z * z, pc, fmaf(-0.5f, z, 1.0f));
  return o;
}

SKT_HD SinCosF sincos_fast(double x, bool* ok) {
  const double invpio2 = 6.36619772367581382433e-01;
  const double pio2_1 = 1.57079632673412561417e+00;  // sincos_bf's constants
  const double pio2_2 = 6.07710050630396597660e-11;
  *ok = fabs(x) < 1647099.3291652855;  // false for NaN / inf too
  const double fn = rint(x * invpio2);
  const double y = (x - fn * pio2_1) - fn * pio2_2;
  const SinCosF k = sincos_poly((float)y);
  const int n = (int)(*ok ? fn : 0.0) & 3;  // |fn| < 2^20 when ok
  SinCosF o;
  o.s = (n & 1) ? k.c : k.s;
  o.c = (n & 1) ? k.s : k.c;
  if (n == 1 || n == 2) o.c = -o.c;
  if (n >= 2) o.s = -o.s;
  return o;
}

// sin/cos of r + d from fp32 sin/cos of r (|error| <= SKT_FAST_ERR) and a
// small exact fp32 d (|d| <= pi/4): the angle-addition formulas.  The fast
// tick uses it for a projectile fired this tick, whose rotation is the
// player's rotation plus the look action times 0.25 (Player.py:33-39; the
// fp64 sum's own rounding, <= 3e-14 at |r| <= 500, is far below the bound).
// |error| <= 1.25*SKT_FAST_ERR + 2e-7 =: SKT_ADD_ERR (tests/trig_check.cpp
// measures the maximum against sinl/cosl and checks it stays below half).
#define SKT_ADD_ERR 6.0e-7f

SKT_HD SinCosF sincos_add(SinCosF r, float d) {
  const SinCosF k = sincos_poly(d);
  SinCosF o;
  o.s = fmaf(r.s, k.c, r.c * k.s);
  o.c = fmaf(r.c, k.c, -(r.s * k.s));
  return o;
}

// true iff d is provably not within `eps` of a half-integer, so that
// rint(p - d_exact) == p - rintf(d) for every integer p and every d_exact with
// |d_exact - d| <= eps (false for NaN / inf: the caller takes the exact path)
SKT_HD bool round_safe(float d, float eps) {
  const float t = d - floorf(d);  // exact for |d| < 2^23
  return fabsf(t - 0.5f) > eps;
}

}  // namespace sktrig
