#!/bin/bash
# The -m gpu suite, then the ResNet / Connect4 / Atari bench lines, the Atari one
# under rocprofv3 --kernel-trace --stats (the tree step's average).  Each GPU
# step has its own limit; the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r4b && export TMPDIR=/tmp
O=$R/gpurun_out/r4b
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 ${TEST_TIMEOUT:-800} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
fi
line() { grep '^{' $1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('learner_corrected') or {}; print('$2', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], 'learner', d['learner_steps_per_s'], 'corrected', c.get('learner_steps_per_s'), c.get('step_ms'))"; }
timeout -k 10 400 python bench.py --net resnet --no-cpu > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 1; }
line $O/c2.log config2
timeout -k 10 400 python bench.py --game connect4 --net resnet --no-cpu > $O/c3.log 2>&1 || { tail -20 $O/c3.log; exit 1; }
line $O/c3.log config3
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_atari -o run -- python bench.py --game atari --no-cpu > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 1; }
line $O/c4.log config4
head -6 $O/kt_atari/run_kernel_stats.csv | cut -d, -f1-8
