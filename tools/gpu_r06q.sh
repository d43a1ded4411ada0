#!/bin/bash
# Round 6: the chain launch in 16-step passes (LDS 33.5 KB, 4 waves/SIMD) against HEAD (one 32-step pass,
# 66 KB, 2 waves/SIMD): multi-step learner parity tests on this tree, then learner / train-loop rates and
# kernel-trace stats of both libraries.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r6q && export TMPDIR=/tmp
O=$R/gpurun_out/r6q
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_learner_multi_gpu.py tests/test_train_loop_gpu.py tests/test_dp_train_loop_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for v in prev cur; do
  if [ $v = cur ]; then unset MZ_LIB; else export MZ_LIB=$R/muzero.jl_amd/lib/libmz_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- python bench.py --no-cpu --steps 3 --warmup 1 --pipeline-moves 0 > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  echo "$v $(grep '^{' $O/$v.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('learner', d['learner_steps_per_s'], d['learner_multi']['call_ms'], 'train', (d.get('train_loop') or {}).get('node_expansions_per_s'))")"
  grep -E "mz_learn_chain|mz_learn_multi" $O/kt_$v/run_kernel_stats.csv | cut -d, -f1-4
done
