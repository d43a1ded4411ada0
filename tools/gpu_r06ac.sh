#!/bin/bash
# Round 6 final: the N = 8 rehearsal on the one-GPU box with the final tree (8 gloo ranks on cuda:0: the
# wait-free chain helpers, the train loop's pinned-memory hand-back), FC default line and Connect4 ResNet.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r6ac && export TMPDIR=/tmp
O=$R/gpurun_out/r6ac
MZ_DIST_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 8 --no-cpu --steps 5 --warmup 1 --pipeline-moves 3 \
  --train-moves 5 --learner-steps 10 > $O/gloo8.log 2>&1 || { tail -30 $O/gloo8.log; exit 1; }
grep '^{' $O/gloo8.log | tail -1 > $O/r06ac_gloo8_bench.json
python -c "import json; d=json.load(open('$O/r06ac_gloo8_bench.json')); print(d['n_gpus'], d['value'], d['learner_config']['form'][:60], d['replica_checks'], d['train_loop']['node_expansions_per_s'], d['train_loop']['learner_steps'], d['config']['parallelism'])"
MZ_DIST_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 8 --game connect4 --net resnet --no-cpu --steps 2 --warmup 1 \
  --pipeline-moves 0 --train-moves 2 --learner-steps 4 > $O/gloo8_c4.log 2>&1 || { tail -30 $O/gloo8_c4.log; exit 1; }
grep '^{' $O/gloo8_c4.log | tail -1 > $O/r06ac_gloo8_connect4_resnet_bench.json
python -c "import json; d=json.load(open('$O/r06ac_gloo8_connect4_resnet_bench.json')); print(d['n_gpus'], d['value'], d['replica_checks'], (d.get('train_loop') or {}).get('learner_steps'))"
