"""How det_tanhf's (include/mz_detmath.h) small-|x| polynomial was made, and its exhaustive check.

1. Fit: tanh(x) = x + x³·P(x²) on [0, 0.55], P of degree 4, iteratively reweighted least squares on the
   relative error of tanh (approximation error 0.018 ulp), coefficients rounded to f32.
2. Check: compile det_tanhf itself (gcc, -ffp-contract=off, the header as the engine and the oracle use it)
   and compare every f32 in [2^-12, 9.5] with tanh in f64 rounded to f32; prints the ulp histogram.
Usage: python tools/fit_tanhf.py [--check-only]
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
T, DEG = 0.55, 5

CHECK_C = r"""
#include "mz_detmath.h"
#include <stdio.h>
#include <stdlib.h>
int main(void) {
    unsigned lo = mz_f2u(0.000244140625f), hi = mz_f2u(9.5f);
    long hist[4] = {0}; int worst = 0; float wx = 0;
    for (unsigned u = lo; u <= hi; ++u) {
        float x = mz_u2f(u), ref = (float)tanh((double)x);
        float c = det_tanhf(x), cn = det_tanhf(-x);
        if (mz_f2u(cn) != (mz_f2u(c) ^ 0x80000000u)) { printf("odd symmetry broken at %.9g\n", x); return 1; }
        int d = abs((int)mz_f2u(c) - (int)mz_f2u(ref));
        if (d > worst) { worst = d; wx = x; }
        hist[d < 3 ? d : 3]++;
    }
    printf("worst %d ulp at %.9g; inputs at 0 / 1 / 2 / >2 ulp: %ld %ld %ld %ld\n", worst, wx,
           hist[0], hist[1], hist[2], hist[3]);
    return worst > 2;
}
"""


def fit():
    s = np.linspace(1e-8, T * T, 20000)
    x = np.sqrt(s)
    f = (np.tanh(x) - x) / x ** 3
    w = x ** 3 / np.tanh(x)
    ww = np.ones_like(s)
    for _ in range(30):
        A = np.vander(s, DEG, increasing=True) * (w * ww)[:, None]
        c = np.linalg.lstsq(A, f * w * ww, rcond=None)[0]
        e = np.abs((np.vander(s, DEG, increasing=True) @ c - f) * w)
        ww *= (e / e.max()) ** 0.3 + 1e-3
    print(f"approximation error {e.max() / 2 ** -24:.4f} ulp; f32 coefficients (x^3 first):",
          [float(v) for v in c.astype(np.float32)])


def check():
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "chk.c"), os.path.join(d, "chk")
        open(src, "w").write(CHECK_C)
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-I", os.path.join(ROOT, "include"), "-o", exe, src,
                        "-lm"], check=True)
        return subprocess.run([exe]).returncode


if __name__ == "__main__":
    if "--check-only" not in sys.argv:
        fit()
    sys.exit(check())
