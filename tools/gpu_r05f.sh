#!/bin/bash
# Round 5: downsampler variant check — parity of the Atari nets, then per-layer stamps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r5f && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_atari_gpu.py \
  > gpurun_out/r5f/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/r5f/tests.log; exit 1; }
tail -1 gpurun_out/r5f/tests.log
MZ_LIB=$R/muzero.jl_amd/lib/libmz_stamps.so timeout -k 10 120 python tools/ds_stamps.py 32 2>&1 | grep -v amdgpu.ids | tail -22
