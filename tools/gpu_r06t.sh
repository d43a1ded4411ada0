#!/bin/bash
# Round 6: mz_learn_chain's helper workgroups (the prediction net's 540 parameters past the slices' first
# pass, one per helper thread, so no slice thread runs two 32-step chains in sequence; the one-parameter
# diagnostic measured 34.0 -> 24.1 us per chain).  Parity: the multi-step learner / train-loop tests
# (helpers on by default for the FC nets; the ResNet cases also with MZ_CHAIN_HELP=1); then learner rates and
# kernel stats of HEAD (prev) and this tree, and the ResNet learner with the helpers forced on and off.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r6t && export TMPDIR=/tmp
O=$R/gpurun_out/r6t
T="tests/test_learner_multi_gpu.py tests/test_train_loop_gpu.py tests/test_dp_train_loop_gpu.py tests/test_fault_gpu.py"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $T > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
MZ_CHAIN_HELP=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_learner_multi_gpu.py > $O/tests_help1.log 2>&1 || { tail -30 $O/tests_help1.log; exit 1; }
tail -2 $O/tests_help1.log
for v in prev cur; do
  if [ $v = cur ]; then unset MZ_LIB; else export MZ_LIB=$R/muzero.jl_amd/lib/libmz_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- python bench.py --no-cpu --steps 3 --warmup 1 --pipeline-moves 0 > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  echo "$v $(grep '^{' $O/$v.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('learner', d['learner_steps_per_s'], d['learner_multi']['call_ms'], 'train', (d.get('train_loop') or {}).get('node_expansions_per_s'))")"
  grep -E "mz_learn_chain|mz_learn_multi" $O/kt_$v/run_kernel_stats.csv | cut -d, -f1-4
done
unset MZ_LIB
for hv in 0 1; do
  MZ_CHAIN_HELP=$hv timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_rn$hv -o run -- python bench.py --net resnet --no-cpu --steps 2 --warmup 1 --pipeline-moves 0 --train-moves 0 > $O/rn$hv.log 2>&1 || { tail -20 $O/rn$hv.log; exit 1; }
  echo "resnet help=$hv $(grep '^{' $O/rn$hv.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('learner', d['learner_steps_per_s'])")"
  grep -E "mz_learn_chain" $O/kt_rn$hv/run_kernel_stats.csv | cut -d, -f1-4
done
