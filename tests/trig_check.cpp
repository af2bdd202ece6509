// CPU check of the step kernels' trig (skillshot_learning_amd/csrc/sk_trig.hpp,
// compiled here for the host with the same -ffp-contract=off; the device
// code evaluates the same IEEE operations, fmaf = v_fma_f32, rint = v_rndne).
//   sincos_bf   : |error| <= 1 ulp against glibc sin/cos (the reference's
//                 math.sin / math.cos), exact at +-0
//   sincos_fast : |error| <= SKT_FAST_ERR / 2 against long-double sinl/cosl
//   sincos_add  : |error| <= SKT_ADD_ERR / 2 (rotation after a look step)
// Prints one line "max_ulp_bf=<u> max_err_fast=<e> n=<count>" and exits 1 on
// a violation.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../skillshot_learning_amd/csrc/sk_trig.hpp"

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint64_t next() {
  rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
  return rng;
}
static double uni(double lo, double hi) { return lo + (hi - lo) * ((next() >> 11) * 0x1p-53); }

static long long ulps(double a, double b) {
  int64_t ia, ib;
  memcpy(&ia, &a, 8); memcpy(&ib, &b, 8);
  if (ia < 0) ia = INT64_MIN - ia;
  if (ib < 0) ib = INT64_MIN - ib;
  long long d = (long long)(ia - ib);
  return d < 0 ? -d : d;
}

static long long max_ulp = 0;
static double max_err = 0, max_err_add = 0;
static long n = 0, fails = 0;

static void check(double x) {
  bool ok1, ok2;
  sktrig::SinCos b = sktrig::sincos_bf(x, &ok1);
  sktrig::SinCosF f = sktrig::sincos_fast(x, &ok2);
  if (!ok1 || !ok2) return;
  ++n;
  long long u = ulps(b.s, sin(x));
  long long v = ulps(b.c, cos(x));
  if (u > max_ulp) max_ulp = u;
  if (v > max_ulp) max_ulp = v;
  long double sx = sinl((long double)x), cx = cosl((long double)x);
  double es = fabs((double)((long double)f.s - sx)), ec = fabs((double)((long double)f.c - cx));
  if (es > max_err) max_err = es;
  if (ec > max_err) max_err = ec;
  // angle addition with a look step d = a*0.25, a an f32 action in [-1, 1]
  const float a = (float)uni(-1.0, 1.0);
  const float d = a * 0.25f;
  const double xd = x + (double)d;  // the fp64 rotation after the look
  sktrig::SinCosF g = sktrig::sincos_add(f, d);
  long double sxd = sinl((long double)xd), cxd = cosl((long double)xd);
  double ea = fabs((double)((long double)g.s - sxd)), eb = fabs((double)((long double)g.c - cxd));
  if (ea > max_err_add) max_err_add = ea;
  if (eb > max_err_add) max_err_add = eb;
  if (ea > SKT_ADD_ERR / 2 || eb > SKT_ADD_ERR / 2) {
    if (fails++ < 10) printf("FAIL add x=%.17g d=%.9g err_s=%g err_c=%g\n", x, (double)d, ea, eb);
  }
  if (u > 1 || v > 1 || es > SKT_FAST_ERR / 2 || ec > SKT_FAST_ERR / 2) {
    if (fails++ < 10) printf("FAIL x=%.17g ulp_s=%lld ulp_c=%lld err_s=%g err_c=%g\n", x, u, v, es, ec);
  }
}

int main(int argc, char** argv) {
  long count = argc > 1 ? atol(argv[1]) : 2000000;
  check(0.0); check(-0.0);
  for (long i = 0; i < count; ++i) check(uni(-600.0, 600.0));          // game rotations (|r| <= 500)
  for (long i = 0; i < count / 4; ++i) check(uni(-4.0, 4.0));
  for (long i = 0; i < count / 4; ++i) check(uni(-1.6e6, 1.6e6));      // whole fast range
  for (long k = -400; k <= 400; ++k)                                   // next to multiples of pi/4
    for (int j = -3; j <= 3; ++j) {
      double c = k * (M_PI / 4);
      check(c + j * 1e-9); check(nextafter(c, 1e9)); check(nextafter(c, -1e9));
    }
  for (long i = 0; i < count / 4; ++i) check(0.25 * (double)(int64_t)(next() % 4001) - 500.0 + 0.25 * uni(-1, 1));
  printf("max_ulp_bf=%lld max_err_fast=%.3e max_err_add=%.3e n=%ld\n", max_ulp, max_err, max_err_add, n);
  return fails ? 1 : 0;
}
