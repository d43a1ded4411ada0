#!/bin/bash
# Round 5, first pass: the multi-step learner's parity tests, the learner /
# train-loop tests they share code with, then one default bench line and the
# kernel stats of the default command.  Each GPU step has its own limit; the
# script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r5a && export TMPDIR=/tmp
O=$R/gpurun_out/r5a
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_learner_multi_gpu.py tests/test_train_loop_gpu.py tests/test_selfplay_gpu.py tests/test_fc_bn.py tests/test_fault_gpu.py tests/test_atari_gpu.py \
  > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/r05a_default_bench.json
python -c "import json; d=json.load(open('$O/r05a_default_bench.json')); print(d['value'], d['learner_steps_per_s'], d['learner_steps_per_s_1step'], d['learner_multi'], d['train_loop']['node_expansions_per_s'], d['train_loop']['learner_steps_per_s'], d['learner_roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python bench.py --no-cpu > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
cp $O/kt/run_kernel_stats.csv $O/r05a_default_kernel_stats.csv
head -12 $O/r05a_default_kernel_stats.csv | cut -d, -f1-8
