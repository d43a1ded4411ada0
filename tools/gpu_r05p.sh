#!/bin/bash
# Round 5: 32-step ADAM chains (the bank halves hold 32 images; unroll launches stay at 16 steps) —
# multi-step / train-loop parity, then alternating learner lines (FC default, TicTacToe ResNet) vs HEAD.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r5p && export TMPDIR=/tmp
O=$R/gpurun_out/r5p
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_learner_multi_gpu.py tests/test_train_loop_gpu.py tests/test_fault_gpu.py > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
b() {
  local n=$1; shift
  timeout -k 10 300 env "$@" > $O/$n.log 2>&1 || { echo "BENCH FAILED $n"; tail -20 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log | tail -1 > $O/$n.json
  python -c "import json; d=json.load(open('$O/$n.json')); m=d['learner_multi'] or {}; t=d['train_loop'] or {}; print('$n', m.get('learner_steps_per_s'), m.get('call_ms'), m.get('steps_per_unroll_launch'), t.get('node_expansions_per_s'), t.get('learner_steps_per_s'))"
}
for rep in 1 2; do
  b fc_new_$rep python bench.py --no-cpu --pipeline-moves 0 --steps 5
  b fc_head_$rep MZ_LIB=$R/muzero.jl_amd/lib/libmz_head.so python bench.py --no-cpu --pipeline-moves 0 --steps 5
  b rn_new_$rep python bench.py --no-cpu --pipeline-moves 0 --steps 5 --net resnet
  b rn_head_$rep MZ_LIB=$R/muzero.jl_amd/lib/libmz_head.so python bench.py --no-cpu --pipeline-moves 0 --steps 5 --net resnet
done
