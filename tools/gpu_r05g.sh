#!/bin/bash
# Round 5: ResNet multi-step learner parity (TicTacToe / Connect4 / Atari-like) + the Atari and
# ResNet learner tests, then learner throughput of the multi-step form on configs[2]/[3]/[4].
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r5g && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_learner_multi_gpu.py tests/test_atari_gpu.py tests/test_fault_gpu.py \
  > gpurun_out/r5g/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/r5g/tests.log; exit 1; }
tail -3 gpurun_out/r5g/tests.log
