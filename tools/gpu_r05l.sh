#!/bin/bash
# Round 5: Dense outputs kept as k-quarter partials, combined by their consumers (mz_small.hip) —
# parity of every small-kernel path (searches small1/2/4 incl. the exact configs[1] launch, FC +
# BatchNorm, the learners one-step / multi-step, the actor-learner loop), then an alternating A/B of
# the default bench line against HEAD's library (libmz_head.so).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r5l && export TMPDIR=/tmp
O=$R/gpurun_out/r5l
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_golden.py tests/test_fc_bn.py tests/test_bench_sizes_gpu.py \
  tests/test_learner_multi_gpu.py tests/test_selfplay_gpu.py tests/test_train_loop_gpu.py \
  > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
b() {  # name, env..., -- args
  local n=$1; shift
  timeout -k 10 300 env "$@" > $O/$n.log 2>&1 || { echo "BENCH FAILED $n"; tail -20 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log | tail -1 > $O/$n.json
  python -c "import json; d=json.load(open('$O/$n.json')); m=d['learner_multi'] or {}; print('$n', d['value'], d['roofline']['kernel_ms'], d['learner_steps_per_s_1step'], m.get('learner_steps_per_s'), (d['train_loop'] or {}).get('node_expansions_per_s'))"
}
for rep in 1 2; do
  b new_$rep python bench.py --no-cpu
  b head_$rep MZ_LIB=$R/muzero.jl_amd/lib/libmz_head.so python bench.py --no-cpu
done
