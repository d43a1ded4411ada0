#!/bin/bash
# Round 5: the ResNet multi-step learner in bench (configs[2] TicTacToe ResNet, configs[3] Connect4
# ResNet, configs[4] Atari-like): multi vs one-step learner steps/s, Ls sweep, kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r5h && export TMPDIR=/tmp
O=$R/gpurun_out/r5h
b() {  # name, args...
  local n=$1; shift
  timeout -k 10 240 python bench.py --no-cpu --pipeline-moves 0 --steps 5 --train-moves 0 "$@" > $O/$n.log 2>&1 || { echo "FAILED $n"; tail -8 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log | tail -1 > $O/$n.json
  python -c "
import json; d=json.load(open('$O/$n.json')); m=d['learner_multi'] or {}; r=d['learner_roofline'] or {}
print('$n', 'multi', m.get('learner_steps_per_s'), 'unroll_ms', m.get('unroll_launch_ms'), 'per_launch', m.get('steps_per_unroll_launch'),
      '1step', d['learner_steps_per_s_1step'], 'frac', r.get('frac'), m.get('kernels'))"
}
b ttt_rn --net resnet
MZ_MULTI_LS=8 b ttt_rn_ls8 --net resnet
MZ_MULTI_LS=4 b ttt_rn_ls4 --net resnet
b c4_rn --game connect4 --net resnet
b atari --game atari
b ttt_rn_b2048 --net resnet --batch 2048 --learner-steps 10 --learner-chunk 16
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python bench.py --no-cpu --pipeline-moves 0 --steps 5 --train-moves 0 --net resnet > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
head -12 $O/kt/run_kernel_stats.csv | cut -d, -f1-5
