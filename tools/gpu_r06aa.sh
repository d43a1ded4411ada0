#!/bin/bash
# Round 6: mz_learn_chain's ADAM step with 1 − β^t formed on the host and each step's constants read one step
# ahead (their LDS reads were on the step's dependent chain), and the first parameter's Σθ² partial stored
# instead of read-modify-written.  Parity tests, then learner / train-loop rates and chain kernel time against
# HEAD (prev), alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r6aa && export TMPDIR=/tmp
O=$R/gpurun_out/r6aa
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_learner_multi_gpu.py tests/test_train_loop_gpu.py tests/test_dp_train_loop_gpu.py tests/test_resnet_gpu.py tests/test_atari_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="--no-cpu --steps 3 --warmup 1 --pipeline-moves 0 --learner-steps 20 --train-moves 30"
for v in prev cur prev2 cur2; do
  if [ ${v%2} = prev ]; then export MZ_LIB=$R/muzero.jl_amd/lib/libmz_prev.so; else unset MZ_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- python bench.py $B > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  echo "$v $(grep '^{' $O/$v.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['train_loop']; print('learner', d['learner_steps_per_s'], 'train', t['node_expansions_per_s'])")"
  grep -E "mz_learn_chain" $O/kt_$v/run_kernel_stats.csv | cut -d, -f1-4
done
