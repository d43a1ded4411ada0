#!/bin/bash
# Round 5: multi-step learner — parity tests, then bench lines by call length.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r5b && export TMPDIR=/tmp
O=$R/gpurun_out/r5b
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_learner_multi_gpu.py tests/test_train_loop_gpu.py tests/test_selfplay_gpu.py > $O/tests.log 2>&1 \
  || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
b() {  # name, env, args
  local n=$1 e=$2; shift 2
  env $e timeout -k 10 200 python bench.py --no-cpu --pipeline-moves 0 --steps 5 "$@" > $O/$n.log 2>&1 || { echo "FAILED $n"; tail -5 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log | tail -1 > $O/$n.json
  python -c "import json; d=json.load(open('$O/$n.json')); m=d['learner_multi'] or {}; t=d['train_loop'] or {}; print('$n', m.get('learner_steps_per_s'), m.get('call_ms'), m.get('unroll_launch_ms'), m.get('steps_per_unroll_launch'), d['learner_steps_per_s_1step'], t.get('node_expansions_per_s'), t.get('learner_steps_per_s'), d['learner_roofline']['frac'])"
}
b L8 X=1 --learner-chunk 8
b L16 X=1 --learner-chunk 16
b L64 X=1
b L128 X=1 --learner-chunk 128
b L64_ls8 MZ_MULTI_LS=8 MZ_MULTI_T=1
