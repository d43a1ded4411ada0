"""The ResNet kernels divide by the BatchNorm denominator s = sqrtf(1+1e-5)
with a reciprocal + two-fma correction (mz_resnet.hip rn_epilogue).  Exhaustive
over all float encodings with |x| >= 2^-100: identical to IEEE x / s (the
oracle's division); smaller |x| take the IEEE division in the kernel."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bn_division_exhaustive(tmp_path):
    exe = tmp_path / "check_bn_div"
    subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", "-o", str(exe),
                    os.path.join(ROOT, "tools", "check_bn_div.c"), "-lm"], check=True)
    out = subprocess.run([str(exe), "1"], check=True, capture_output=True, text=True,
                         env={**os.environ, "OMP_NUM_THREADS": str(min(8, os.cpu_count() or 1))}).stdout
    assert out.split()[-1] == "0", out
