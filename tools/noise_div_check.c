/* Exhaustive check of the noise3d division shortcut (dt_kernels.hip noise3d):
 * for every integer x in [0, 2^31) -- the range of noise.h's masked hash t -- the
 * Markstein sequence q0 = RN(x*r), e = fma(-c, q0, x), q = fma(e, r, q0) with r = RN(1/c)
 * equals the correctly rounded x / c, c = 1073741823 (noise.h:43). Prints the mismatch
 * count (0 expected).  gcc -O2 -fopenmp -ffp-contract=off noise_div_check.c -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>

int main(void)
{
  const double c = 1073741823.0;
  volatile double one = 1.0;
  const double r = one / c;
  long bad = 0;
#pragma omp parallel for reduction(+ : bad) schedule(static)
  for (int64_t i = 0; i < ((int64_t)1 << 31); ++i) {
    const double x = (double)i;
    const double q0 = x * r;
    const double e = fma(-c, q0, x);
    const double q = fma(e, r, q0);
    if (q != x / c) ++bad;
  }
  printf("%ld\n", bad);
  return bad != 0;
}
