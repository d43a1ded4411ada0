#!/bin/bash
# Round 6: the whole -m gpu suite on this tree, then the N = 8 rehearsal on the one-GPU box
# (8 ranks over gloo, all on cuda:0): the multi-step DP learner, the DP train loop, replica checks.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r6f && export TMPDIR=/tmp
O=$R/gpurun_out/r6f
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
MZ_DIST_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 8 --no-cpu --steps 5 --warmup 1 --pipeline-moves 3 \
  --train-moves 5 --learner-steps 10 > $O/gloo8.log 2>&1 || { tail -30 $O/gloo8.log; exit 1; }
grep '^{' $O/gloo8.log | tail -1 > $O/r06f_gloo8_bench.json
python -c "import json; d=json.load(open('$O/r06f_gloo8_bench.json')); print(d['n_gpus'], d['value'], d['learner_config']['form'][:60], d['replica_checks'], d['train_loop']['node_expansions_per_s'], d['train_loop']['learner_steps'], d['config']['parallelism'])"
