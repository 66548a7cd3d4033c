"""Degree-11 Chebyshev fit of exp on |r| <= ln2/2 (the coefficients of
nuts_device.hip::exp_poly) and its ulp check against expl (gcc, host).

    python scripts/micro/exp_fit.py
"""
import os
import subprocess
import tempfile

import mpmath as mp

mp.mp.dps = 50
H = mp.log(2) / 2
poly, err = mp.chebyfit(mp.exp, [-H, H], 12, error=True)
coef = [repr(float(c)) for c in poly]
print("fit error", mp.nstr(err, 5))
print("coefficients (highest first):", ", ".join(coef))
SRC = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static const double C[] = {%s};
static double ev(double x) {
  const double SH = 6755399441055744.0;
  const double t = fma(x, 1.4426950408889634, SH), n = t - SH;
  double r = fma(-n, 6.93147180369123816490e-01, x);
  r = fma(-n, 1.90821492927058770002e-10, r);
  double p = C[0];
  for (int i = 1; i <= 11; ++i) p = fma(p, r, C[i]);
  return ldexp(p, (int)n);
}
int main(void) {
  uint64_t s = 88172645463325252ull; int64_t m = 0;
  for (long i = 0; i < 20000000; i++) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    const double u = (double)(s >> 11) * 0x1.0p-53, x = (i & 1) ? -u : -60.0 * u;
    const double v = ev(x), ref = (double)expl((long double)x);
    int64_t a, b; memcpy(&a, &v, 8); memcpy(&b, &ref, 8);
    if (llabs(a - b) > m) m = llabs(a - b);
  }
  printf("max ulp vs correctly rounded exp over 2e7 points in [-60, 0]: %%ld\n", (long)m);
  return 0;
}
""" % ", ".join(coef)
with tempfile.TemporaryDirectory() as d:
    c, exe = os.path.join(d, "t.c"), os.path.join(d, "t")
    open(c, "w").write(SRC)
    subprocess.check_call(["gcc", "-O2", "-o", exe, c, "-lm"])
    subprocess.check_call([exe])
