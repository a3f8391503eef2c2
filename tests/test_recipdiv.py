"""Host check of the shared-divisor quotient the Gaussian models use (bates_gauss.h RecipDiv):
with y = RN(1/b), q = RN(a*y), r = fma(-q, b, a), t = fma(r, y, q) equals the IEEE quotient
a/b bit for bit inside the kernel's guard (|b| in [2^-500, 2^500], |a| in [2^-900, 2^401])
-- Markstein's theorem, checked here on random and adversarial operands with the host's fma."""
import os
import shutil
import subprocess
import tempfile

import pytest

SRC = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint64_t nx(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double mk(int emin, int emax, int allones) {
  uint64_t m = nx() & ((1ull << 52) - 1);
  if (allones) m = ((1ull << 52) - 1) ^ (nx() & 7);   /* significands near 2 - ulp */
  int e = emin + (int)(nx() % (uint64_t)(emax - emin + 1));
  uint64_t bits = ((uint64_t)(e + 1023) << 52) | m | ((nx() & 1) << 63);
  double d; memcpy(&d, &bits, 8); return d;
}
int main(int argc, char** argv) {
  long n = atol(argv[1]), bad = 0;
  for (long i = 0; i < n; ++i) {
    const int mode = (int)(i % 4);
    double b = mk(-500, 499, mode == 1);
    double a = mk(-900, 400, mode == 2);
    if (mode == 3) { b = mk(-3, 3, 0); a = mk(-2, 8, 0); }   /* the fits' usual range */
    if (argc > 2) {  /* the DM models' constant divisors (div_const): 1374^3, 135^3 */
      b = strtod(argv[2], 0);
      a = (i & 1) ? mk(-900, 900, 0) : mk(20, 40, 0);
    }
    volatile double y = 1.0 / b;
    volatile double q = a * y;
    volatile double r = fma(-q, b, a);
    volatile double t = fma(r, y, q);
    volatile double ref = a / b;
    if (memcmp((const void*)&t, (const void*)&ref, 8) != 0) {
      if (bad < 5) printf("mismatch a=%a b=%a t=%a ref=%a\n", a, b, t, ref);
      ++bad;
    }
  }
  printf("%ld %ld\n", n, bad);
  return bad != 0;
}
"""


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_shared_divisor_quotient_is_correctly_rounded():
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "rd.c")
        exe = os.path.join(d, "rd")
        open(c, "w").write(SRC.replace("#include <string.h>", "#include <string.h>\n#include <stdlib.h>"))
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", c, "-o", exe, "-lm"], check=True)
        out = subprocess.run([exe, "4000000"], capture_output=True, text=True, timeout=120)
        assert out.returncode == 0, out.stdout
        n, bad = map(int, out.stdout.split()[-2:])
        assert n == 4000000 and bad == 0
        # div_const of the DM-curve models (bates_common.h): PHCX F3 = 1374^3, PFD 135^3,
        # |a| in [2^-900, 2^900]
        for f3 in ("2593941624", "2460375"):
            out = subprocess.run([exe, "4000000", f3], capture_output=True, text=True, timeout=120)
            assert out.returncode == 0, out.stdout
            n, bad = map(int, out.stdout.split()[-2:])
            assert n == 4000000 and bad == 0
