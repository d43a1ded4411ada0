#!/bin/bash
# Round 5: the whole -m gpu suite after the ResNet multi-step learner, then the ResNet train loop
# (mz_train_run now chunks ResNet learner steps too) on configs[2] and configs[4].
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r5i && export TMPDIR=/tmp
O=$R/gpurun_out/r5i
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests \
  > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for cfg in "--net resnet" "--game atari" "--game connect4 --net resnet"; do
  n=$(echo $cfg | tr -d ' -')
  timeout -k 10 300 python bench.py --no-cpu $cfg > $O/$n.log 2>&1 || { echo "BENCH FAILED $cfg"; tail -20 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log | tail -1 > $O/r05i_$n.json
  python -c "import json; d=json.load(open('$O/r05i_$n.json')); t=d['train_loop']; print('$n', d['value'], d['learner_steps_per_s'], d['learner_steps_per_s_1step'], t['node_expansions_per_s'], t['learner_steps_per_s'], d['selfplay_pipeline'] and d['selfplay_pipeline'].get('node_expansions_per_s'))"
done
