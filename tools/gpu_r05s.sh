#!/bin/bash
# Round 5 experiment: FC multi-step unroll launches of 32 steps (two workgroup rounds per CU) vs 16.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r5s && export TMPDIR=/tmp
O=$R/gpurun_out/r5s
b() {
  local n=$1; shift
  timeout -k 10 300 env "$@" > $O/$n.log 2>&1 || { echo "BENCH FAILED $n"; tail -20 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log | tail -1 > $O/$n.json
  python -c "import json; d=json.load(open('$O/$n.json')); m=d['learner_multi'] or {}; print('$n', m.get('learner_steps_per_s'), m.get('call_ms'), m.get('steps_per_unroll_launch'), m.get('unroll_launch_ms'))"
}
for rep in 1 2; do
  b ls16_$rep python bench.py --no-cpu --pipeline-moves 0 --steps 3 --train-moves 0
  b ls32_$rep MZ_MULTI_LS=32 python bench.py --no-cpu --pipeline-moves 0 --steps 3 --train-moves 0
  b ls24_$rep MZ_MULTI_LS=24 python bench.py --no-cpu --pipeline-moves 0 --steps 3 --train-moves 0
done
