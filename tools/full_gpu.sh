#!/bin/bash
# Round-end rehearsal: the whole -m gpu suite, smoke(), then the default bench line.
# Each GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
