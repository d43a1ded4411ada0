#!/bin/bash
# FC corrected learner after BP_SKIP + batched dW / db loads: parity tests, the
# corrected leg (3 runs) and its kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/${TAG:-r05u}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_corrected_learner_gpu.py tests/test_dp_libmz_gpu.py tests/test_corrected_resnet_gpu.py > gpurun_out/${TAG:-r05u}/tests.log 2>&1 || { tail -30 gpurun_out/${TAG:-r05u}/tests.log; exit 1; }
tail -2 gpurun_out/${TAG:-r05u}/tests.log
LIBS="${LIBS:-base base base}" bash tools/ab_corrected.sh || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG:-r05u}/prof -o run -- python bench.py --no-cpu --steps 2 --warmup 1 --pipeline-moves 0 --train-moves 0 --learner-steps 40 > gpurun_out/${TAG:-r05u}/prof.log 2>&1 || { tail -20 gpurun_out/${TAG:-r05u}/prof.log; exit 1; }
f=$(find gpurun_out/${TAG:-r05u}/prof -name '*kernel_stats.csv' | head -1); grep -E "bp_|adam" "$f" | cut -c1-160
