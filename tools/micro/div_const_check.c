/* Host check of div_const (csrc/usv_device.hpp): for each compile-time divisor c of the f64 build,
 * q = RN(x y) with y = RN(1 / c), r = x - q c (one fma, exact), RN(q + r y) must equal the IEEE quotient
 * x / c.  Random operands with random sign, mantissa and exponent in [-60, 60].
 *   gcc -O2 -o div_const_check div_const_check.c -lm && ./div_const_check [samples per divisor]
 * Exit status 0 iff no mismatch. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s = 88172645463325252ull;
static uint64_t xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 10000000L;
  volatile double iz = 4.1, nrd = -2.79, m = 30.0, xud = -2.25, b = 0.41, cth = 0.78;
  const double cs[] = {0.01, m - xud, iz - nrd, b, 2 * cth, b * cth,            /* ASMC substep */
                       10.0, 3.14159265358979323846, 28.284271247461902, 0.075}; /* header, reward */
  long bad_total = 0;
  for (unsigned k = 0; k < sizeof(cs) / sizeof(cs[0]); ++k) {
    const double c = cs[k], y = 1.0 / c;
    long bad = 0, plain = 0;
    for (long i = 0; i < n; ++i) {
      uint64_t bits = xr();
      bits = (bits & 0x800FFFFFFFFFFFFFull) | ((uint64_t)(1023 - 60 + (xr() % 121)) << 52);
      double x;
      memcpy(&x, &bits, 8);
      const double q = x * y;
      const double q1 = fma(fma(-q, c, x), y, q);
      bad += q1 != x / c;
      plain += q != x / c;
    }
    printf("c = %.17g: %ld mismatches of %ld (a plain multiply by 1/c: %ld)\n", c, bad, n, plain);
    bad_total += bad;
  }
  return bad_total != 0;
}
