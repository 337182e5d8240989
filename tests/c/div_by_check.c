/* CPU check of the env kernel's division by the normaliser count (t2o_env.hip
 * div_by): q = a*y with y = RN(1/n), then two fma residual corrections, against
 * IEEE a/n.  Inputs: the normaliser's operand families (differences of grid
 * values, integers, random doubles over a wide exponent range), n up to argv[1].
 * Prints the number of mismatches (expected 0).  Built and run by
 * tests/test_env_division.py. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s = 88172645463325252ull;
static uint64_t xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double ud(void) { return (double)(xr() >> 11) * 0x1.0p-53; }

static double div_by(double a, double n, double y) {
  double q = a * y;
  double r = fma(-q, n, a);
  q = fma(r, y, q);
  r = fma(-q, n, a);
  return fma(r, y, q);
}

int main(int argc, char** argv) {
  const long nmax = argc > 1 ? atol(argv[1]) : 20000;
  const int per = argc > 2 ? atoi(argv[2]) : 100;
  long bad = 0, total = 0;
  for (long n = 2; n <= nmax; ++n) {
    const double dn = (double)n, y = 1.0 / dn;
    for (int k = 0; k < per; ++k) {
      double a;
      switch (xr() % 4) {
        case 0: a = ud() * 1000.0 - 500.0; break;                                  /* x - mean */
        case 1: a = (double)(int64_t)(xr() % 2000001) - 1000000.0; break;          /* integers */
        case 2: a = (ud() - 0.5) * ldexp(1.0, (int)(xr() % 200) - 100); break;     /* exponents */
        default: a = (double)(int64_t)(xr() % 100001) / 100.0 - ud() * 100.0; break; /* hundredths */
      }
      const double r = a / dn, q = div_by(a, dn, y);
      if (memcmp(&r, &q, 8) != 0) ++bad;
      ++total;
    }
  }
  printf("%ld %ld\n", bad, total);
  return 0;
}
