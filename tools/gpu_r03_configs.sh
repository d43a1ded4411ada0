#!/bin/bash
# One clean bench line per BASELINE config (no profiler): configs[1] (the default), configs[0]
# (one game x 25 sims), configs[2] (TicTacToe ResNet 2048 games), configs[3] (Connect4
# ResNet-8 512 games/GPU), configs[4] (Atari-like, 200 sims).  Each step has its own limit;
# the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/cfg && export TMPDIR=/tmp
O=gpurun_out/cfg; T=${TAG:-rXX}
run() {  # name, limit, bench args...
  local n=$1 l=$2; shift 2
  timeout -k 10 $l python bench.py "$@" > $O/$n.log 2>&1 || { echo "FAILED $n"; tail -20 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log | tail -1 > $O/${T}_${n}_bench.json
  python -c "import json,sys; d=json.load(open('$O/${T}_${n}_bench.json')); print('$n', d['value'], d.get('learner_steps_per_s'), d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'))"
}
run config1 300
run config0 200 --games 1 --sims 25 --learner-steps 50 --train-moves 0
run config2 400 --net resnet
run config3 400 --game connect4 --net resnet
run config4 400 --game atari
