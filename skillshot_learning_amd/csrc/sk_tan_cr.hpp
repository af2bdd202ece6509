// sk_tan_cr.hpp — correctly rounded fp64 tan (host- and device-compilable).
//
// Why: the future-collision flag (SkillshotGame.check_future_collision,
// SkillshotGame.py:96-113; obs[11]) compares g*X + (qy - g*qx) against the
// opponent's y span with g = math.tan(-rot + pi/2) (Projectile.py:58).  The
// probe boards (tests/golden/make_probes.py) put that value on the span's edge
// up to fp64 rounding, where a 1-ulp difference in g flips the flag: ocml's tan
// differs from glibc's in ~9 % of arguments and flipped 21 of 12000 probe
// flags.  The step kernels keep their fast tan and decide the flag from it
// unless the compare lies within an error margin of an edge; only those lanes
// call tan_cr and redo the compare in the reference's operation order.
//
// Parity bar this buys: glibc 2.35's tan (the reference's math.tan) is itself
// not correctly rounded — 523 of 200800 arguments measured against a 70-digit
// Decimal tan differ by 1 ulp — so the flag equals the reference's wherever
// glibc's tan is correctly rounded, and equals the decision under the correctly
// rounded tan where it is not (tests/golden/probes.npz stores both).
//
// Algorithm: k = rint(x * 2/pi); r = x - k*pi/2 in double-double with pi/2
// split in three doubles (the first product split exactly by fma, x - k*P1
// exact by Sterbenz); sin r and cos r by their Taylor series to r^29 in
// double-double, Horner in r^2 over tabulated double-double coefficients (no
// divisions; |r| <= pi/4: truncation < 2^-110); tan = sin/cos for even k,
// -cos/sin for odd k; the double-double quotient rounded once.  Relative error
// before the final rounding is ~2^-95, so the result is the correctly rounded
// tan except within 2^-95 of a rounding midpoint.  |x| >= 2^20 is handed to
// the platform tan (game rotations stay far below).  Compile with
// -ffp-contract=off: the error-free transformations need separately rounded
// operations (fma is called explicitly where it is wanted).
#pragma once
#include <math.h>

#if defined(__HIPCC__)
#define SKTC_HD __host__ __device__ __forceinline__
#define SKTC_NOINLINE __host__ __device__ __forceinline__
#else
#define SKTC_HD static inline
#define SKTC_NOINLINE static
#endif

namespace sktan {

struct DD {
  double h, l;
};

SKTC_HD DD quick_two_sum(double a, double b) {
  double s = a + b;
  return {s, b - (s - a)};
}
SKTC_HD DD two_sum(double a, double b) {
  double s = a + b;
  double bb = s - a;
  return {s, (a - (s - bb)) + (b - bb)};
}
SKTC_HD DD two_prod(double a, double b) {
  double p = a * b;
  return {p, fma(a, b, -p)};
}
SKTC_HD DD add(DD a, DD b) {
  DD s = two_sum(a.h, b.h), t = two_sum(a.l, b.l);
  s.l += t.h;
  s = quick_two_sum(s.h, s.l);
  s.l += t.l;
  return quick_two_sum(s.h, s.l);
}
SKTC_HD DD neg(DD a) { return {-a.h, -a.l}; }
SKTC_HD DD mul(DD a, DD b) {
  DD p = two_prod(a.h, b.h);
  p.l += a.h * b.l + a.l * b.h;
  return quick_two_sum(p.h, p.l);
}
SKTC_HD DD mul_d(DD a, double b) {
  DD p = two_prod(a.h, b);
  p.l += a.l * b;
  return quick_two_sum(p.h, p.l);
}
SKTC_HD DD div(DD a, DD b) {
  double q1 = a.h / b.h;
  DD r = add(a, neg(mul_d(b, q1)));
  double q2 = r.h / b.h;
  r = add(r, neg(mul_d(b, q2)));
  double q3 = r.h / b.h;
  DD q = quick_two_sum(q1, q2);
  return add(q, DD{q3, 0.0});
}

// pi/2 = P1 + P2 + P3 (+ 5.6e-50)
constexpr double kP1 = 0x1.921fb54442d18p+0;
constexpr double kP2 = 0x1.1a62633145c07p-54;
constexpr double kP3 = -0x1.f1976b7ed8fbcp-110;
constexpr double kTwoOverPi = 0.6366197723675814;

// (-1)^k / (2k+1)! as double-double (hi, lo), k = 0..14
constexpr double kSinC[15][2] = {
    {0x1.0000000000000p+0, 0x0.0p+0},
    {-0x1.5555555555555p-3, -0x1.5555555555555p-57},
    {0x1.1111111111111p-7, 0x1.1111111111111p-63},
    {-0x1.a01a01a01a01ap-13, -0x1.a01a01a01a01ap-73},
    {0x1.71de3a556c734p-19, -0x1.c154f8ddc6c00p-73},
    {-0x1.ae64567f544e4p-26, 0x1.c062e06d1f209p-80},
    {0x1.6124613a86d09p-33, 0x1.f28e0cc748ebep-87},
    {-0x1.ae7f3e733b81fp-41, -0x1.1d8656b0ee8cbp-97},
    {0x1.952c77030ad4ap-49, 0x1.ac981465ddc6cp-103},
    {-0x1.2f49b46814157p-57, -0x1.2650f61dbdcb4p-112},
    {0x1.71b8ef6dcf572p-66, -0x1.d043ae40c4647p-120},
    {-0x1.761b41316381ap-75, 0x1.3423c7d91404fp-130},
    {0x1.3f3ccdd165fa9p-84, -0x1.58ddadf344487p-139},
    {-0x1.d1ab1c2dccea3p-94, -0x1.054d0c78aea14p-149},
    {0x1.259f98b4358adp-103, 0x1.eaf8c39dd9bc5p-157},
};
// (-1)^k / (2k)! as double-double (hi, lo), k = 0..14
constexpr double kCosC[15][2] = {
    {0x1.0000000000000p+0, 0x0.0p+0},
    {-0x1.0000000000000p-1, 0x0.0p+0},
    {0x1.5555555555555p-5, 0x1.5555555555555p-59},
    {-0x1.6c16c16c16c17p-10, 0x1.f49f49f49f49fp-65},
    {0x1.a01a01a01a01ap-16, 0x1.a01a01a01a01ap-76},
    {-0x1.27e4fb7789f5cp-22, -0x1.cbbc05b4fa99ap-76},
    {0x1.1eed8eff8d898p-29, -0x1.2aec959e14c06p-83},
    {-0x1.93974a8c07c9dp-37, -0x1.05d6f8a2efd1fp-92},
    {0x1.ae7f3e733b81fp-45, 0x1.1d8656b0ee8cbp-101},
    {-0x1.6827863b97d97p-53, -0x1.eec01221a8b0bp-107},
    {0x1.e542ba4020225p-62, 0x1.ea72b4afe3c2fp-120},
    {-0x1.0ce396db7f853p-70, 0x1.aebcdbd20331cp-124},
    {0x1.f2cf01972f578p-80, -0x1.9ada5fcc1ab14p-135},
    {-0x1.88e85fc6a4e5ap-89, 0x1.71c37ebd16540p-143},
    {0x1.0a18a2635085dp-98, 0x1.b9e2e28e1aa54p-153},
};

// sum_k C[k] * z^k by Horner in double-double
SKTC_HD DD horner(const double (*C)[2], DD z) {
  DD acc = {C[14][0], C[14][1]};
  for (int k = 13; k >= 0; --k) acc = add(mul(acc, z), DD{C[k][0], C[k][1]});
  return acc;
}

SKTC_NOINLINE double tan_cr(double x) {
  if (!(fabs(x) < 1048576.0)) return tan(x);
  const double k = rint(x * kTwoOverPi);
  const DD p1 = two_prod(k, kP1);
  DD r = two_sum(x - p1.h, -p1.l);  // x - p1.h is exact (Sterbenz)
  r = add(r, neg(two_prod(k, kP2)));
  r = add(r, DD{-(k * kP3), 0.0});
  const DD r2 = mul(r, r);
  const DD s = mul(r, horner(kSinC, r2));
  const DD c = horner(kCosC, r2);
  const long long ki = (long long)k;
  const DD t = (ki & 1) ? neg(div(c, s)) : div(s, c);
  return t.h + t.l;
}

}  // namespace sktan
