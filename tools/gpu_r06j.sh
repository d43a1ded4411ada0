#!/bin/bash
# Round 6: the select-free sequential sum (gseqsum) — the whole -m gpu suite, then an alternating
# A/B of the default bench line against the round-5 library (head).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r6j && export TMPDIR=/tmp
O=$R/gpurun_out/r6j
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in head cur; do
    unset MZ_LIB
    [ $v = head ] && export MZ_LIB=$R/muzero.jl_amd/lib/libmz_head.so
    timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 3 --pipeline-moves 10 --train-moves 10 --learner-steps 30 > $O/ab_${v}_$i.log 2>&1 || { tail -20 $O/ab_${v}_$i.log; exit 1; }
    echo "$v $(tail -1 $O/ab_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['train_loop']; print('exp/s', round(d['value']/1e6,2), d['roofline']['kernel_ms'], 'learner', d['learner_steps_per_s'], d['learner_steps_per_s_1step'], 'pipe', round(d['selfplay_pipeline']['node_expansions_per_s']/1e6,2), 'train', round(t['node_expansions_per_s']/1e6,2))")"
  done
done
