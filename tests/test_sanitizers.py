"""Host sanitizer builds: the C oracle and the checkpoint
header reader (muzero.jl_amd/csrc/mz_st_header.h, compiled into libmz's
mz_checkpoint_load) built with -fsanitize=address,undefined by
tests/sanitize/Makefile and run as standalone programs: the oracle on the
actor-learner loop, PER, searches (FC / ResNet / Connect4) and the Atari
downsampler; the reader on malformed, truncated and mutated headers.  Any
sanitizer report fails the run (-fno-sanitize-recover)."""
import os
import shutil
import subprocess

import pytest

SAN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sanitize")


@pytest.fixture(scope="module")
def built():
    if not shutil.which("gcc") or not shutil.which("g++"):
        pytest.skip("no host compiler")
    subprocess.run(["make", "-s", "-C", SAN], check=True)
    return os.path.join(SAN, "_build")


@pytest.mark.parametrize("prog", ["oracle_asan", "ckpt_header_asan"])
def test_sanitizer_build_clean(built, prog):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(built, prog)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr
