#!/bin/bash
# Atari tree-step phase stamps, then the corrected learners: the ResNet
# configs[2] / configs[3] lines and the FC default line under kernel-trace stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r4f && export TMPDIR=/tmp
O=$R/gpurun_out/r4f
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "corrected or resnet_gpu" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python tools/tree_stamps.py --no-build > $O/ts_atari.log 2>&1 || { tail -20 $O/ts_atari.log; exit 1; }
cat $O/ts_atari.log
timeout -k 10 200 python tools/bp_stamps.py > $O/bp_stamps.log 2>&1 || { tail -20 $O/bp_stamps.log; exit 1; }
cat $O/bp_stamps.log
NET=resnet GAME=connect4 timeout -k 10 200 python tools/bp_stamps.py > $O/rbp_stamps.log 2>&1 || { tail -20 $O/rbp_stamps.log; exit 1; }
cat $O/rbp_stamps.log
line() { grep '^{' $1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('learner_corrected') or {}; print('$2', d['value'], d['roofline']['frac'], 'learner', d['learner_steps_per_s'], 'corrected', c.get('learner_steps_per_s'), c.get('step_ms'))"; }
for c in default resnet connect4; do
  case $c in default) A="";; resnet) A="--net resnet";; connect4) A="--game connect4 --net resnet";; esac
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$c -o run -- python bench.py $A --no-cpu > $O/$c.log 2>&1 || { tail -20 $O/$c.log; exit 1; }
  line $O/$c.log $c
  head -14 $O/kt_$c/run_kernel_stats.csv | cut -d, -f1-4
done
