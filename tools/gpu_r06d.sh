#!/bin/bash
# Round 6: alternating A/B of the default bench line over library variants: the round-5 library (head),
# round 5 + the f32 tanh alone (tanh), this tree's library with and without the tail schedule.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r6d && export TMPDIR=/tmp
O=$R/gpurun_out/r6d
for i in 1 2 3; do
  for v in ${VARIANTS:-head tanh tail notail}; do
    unset MZ_LIB MZ_NO_TAIL
    case $v in head|tanh|x*) export MZ_LIB=$R/muzero.jl_amd/lib/libmz_$v.so;; esac
    [ $v = notail ] && export MZ_NO_TAIL=1
    timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 3 --pipeline-moves 10 --train-moves 0 --learner-steps 30 > $O/ab_${v}_$i.log 2>&1 || { tail -20 $O/ab_${v}_$i.log; exit 1; }
    echo "$v $(tail -1 $O/ab_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('exp/s', round(d['value']/1e6,2), d['roofline']['kernel'], d['roofline']['kernel_ms'], 'learner', d['learner_steps_per_s'], d['learner_steps_per_s_1step'], 'pipe', round(d['selfplay_pipeline']['node_expansions_per_s']/1e6,2))")"
  done
done
