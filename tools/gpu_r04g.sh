#!/bin/bash
# The -m gpu suite, the ResNet corrected learner's application stamps
# (Connect4), then the configs[2] / configs[3] / configs[4] lines under
# kernel-trace stats.  Each GPU step has its own limit; stop at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r4g && export TMPDIR=/tmp
O=$R/gpurun_out/r4g
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 ${TEST_TIMEOUT:-800} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
fi
timeout -k 10 200 python tools/bp_stamps.py > $O/bp_stamps.log 2>&1 || { tail -20 $O/bp_stamps.log; exit 1; }
cat $O/bp_stamps.log
NET=resnet GAME=connect4 timeout -k 10 200 python tools/bp_stamps.py > $O/rbp_stamps.log 2>&1 || { tail -20 $O/rbp_stamps.log; exit 1; }
cat $O/rbp_stamps.log
line() { grep '^{' $1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('learner_corrected') or {}; print('$2', d['value'], d['roofline']['frac'], 'learner', d['learner_steps_per_s'], 'corrected', c.get('learner_steps_per_s'), c.get('step_ms'))"; }
for c in default resnet connect4 atari; do
  case $c in default) A="";; resnet) A="--net resnet";; connect4) A="--game connect4 --net resnet";; atari) A="--game atari";; esac
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$c -o run -- python bench.py $A --no-cpu > $O/$c.log 2>&1 || { tail -20 $O/$c.log; exit 1; }
  line $O/$c.log $c
  head -10 $O/kt_$c/run_kernel_stats.csv | cut -d, -f1-4
done
