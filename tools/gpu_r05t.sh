#!/bin/bash
# FC corrected learner A/B (BP_SKIP, batched dW / db loads): its parity tests,
# then base / variants alternated, then the kernel stats of the base leg
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r05t
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_corrected_learner_gpu.py tests/test_dp_libmz_gpu.py > gpurun_out/r05t_tests.log 2>&1 || { tail -30 gpurun_out/r05t_tests.log; exit 1; }
tail -2 gpurun_out/r05t_tests.log
LIBS="${LIBS:-base noskip nodw base noskip nodw}" bash tools/ab_corrected.sh || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05t/prof -o run -- python bench.py --no-cpu --steps 2 --warmup 1 --pipeline-moves 0 --train-moves 0 --learner-steps 40 > gpurun_out/r05t/prof.log 2>&1 || { tail -20 gpurun_out/r05t/prof.log; exit 1; }
f=$(find gpurun_out/r05t/prof -name '*kernel_stats.csv' | head -1); grep -E "bp_|adam" "$f" | cut -c1-160
