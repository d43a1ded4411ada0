#!/bin/bash
# The default / ResNet / Connect4 / Atari bench lines under kernel-trace stats
# (corrected-learner leg included).  Each GPU step has its own limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r4h && export TMPDIR=/tmp
O=$R/gpurun_out/r4h
line() { grep '^{' $1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('learner_corrected') or {}; print('$2', d['value'], d['roofline']['frac'], 'learner', d['learner_steps_per_s'], 'corrected', c.get('learner_steps_per_s'), c.get('step_ms'))"; }
for c in ${CONFIGS:-default resnet connect4 atari}; do
  case $c in default) A="";; resnet) A="--net resnet";; connect4) A="--game connect4 --net resnet";; atari) A="--game atari";; esac
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$c -o run -- python bench.py $A --no-cpu > $O/$c.log 2>&1 || { tail -20 $O/$c.log; exit 1; }
  line $O/$c.log $c
  head -10 $O/kt_$c/run_kernel_stats.csv | cut -d, -f1-4
done
