#!/bin/bash
# Tree-step phase stamps (Atari-like, TicTacToe ResNet), then kernel-trace stats
# of the configs[2] and configs[3] lines (search, learner, corrected learner).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r4e && export TMPDIR=/tmp
O=$R/gpurun_out/r4e
timeout -k 10 200 python tools/tree_stamps.py --no-build > $O/ts_atari.log 2>&1 || { tail -20 $O/ts_atari.log; exit 1; }
cat $O/ts_atari.log
GAME=ttt G=2048 timeout -k 10 200 python tools/tree_stamps.py --no-build > $O/ts_ttt.log 2>&1 || { tail -20 $O/ts_ttt.log; exit 1; }
cat $O/ts_ttt.log
for c in resnet connect4; do
  if [ $c = resnet ]; then A="--net resnet"; else A="--game connect4 --net resnet"; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$c -o run -- python bench.py $A --no-cpu --steps 5 --warmup 1 --pipeline-moves 0 > $O/$c.log 2>&1 || { tail -20 $O/$c.log; exit 1; }
  head -14 $O/kt_$c/run_kernel_stats.csv | cut -d, -f1-4
done
