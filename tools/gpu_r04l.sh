#!/bin/bash
# Corrected-learner tests, the FC corrected-learner level stamps (ALAP backward
# levels, L2 warm-up), then the default and Atari lines under kernel-trace stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r4l && export TMPDIR=/tmp
O=$R/gpurun_out/r4l
timeout -k 10 300 python -u -m pytest tests/test_corrected_resnet_gpu.py tests/test_corrected_learner_gpu.py tests/test_fc_bn.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 200 python tools/bp_stamps.py > $O/bp_stamps.log 2>&1 || { tail -20 $O/bp_stamps.log; exit 1; }
cat $O/bp_stamps.log
for c in default atari; do
  case $c in default) A="";; atari) A="--game atari";; esac
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$c -o run -- python bench.py $A --no-cpu > $O/$c.log 2>&1 || { tail -20 $O/$c.log; exit 1; }
  grep '^{' $O/$c.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['learner_steps_per_s'], d['learner_corrected']['learner_steps_per_s'], d['learner_corrected']['step_ms'])"
  head -12 $O/kt_$c/run_kernel_stats.csv | cut -d, -f1-4
done
