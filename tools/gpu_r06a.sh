#!/bin/bash
# Round 6: the tail schedule + f32 tanh — the whole -m gpu suite, then alternating A/B of the default
# bench line with the tail (in-tree library) and without it (MZ_NO_TAIL=1, same library).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r6a && export TMPDIR=/tmp
O=$R/gpurun_out/r6a
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
  > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for v in tail notail; do
    if [ $v = notail ]; then export MZ_NO_TAIL=1; else unset MZ_NO_TAIL; fi
    timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 3 --pipeline-moves 10 --train-moves 0 > $O/ab_${v}_$i.log 2>&1 || { tail -20 $O/ab_${v}_$i.log; exit 1; }
    echo "$v $(tail -1 $O/ab_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('exp/s', round(d['value']/1e6,2), d['roofline']['kernel'], d['roofline']['kernel_ms'], 'learner', d['learner_steps_per_s'], 'pipe', round(d['selfplay_pipeline']['node_expansions_per_s']/1e6,2))")"
  done
done
