#!/bin/bash
# Round 6: 4 samples per unroll workgroup in the multi-step FC learner (mz_learn_multi4, 32 steps per
# unroll launch) — the multi-step parity tests as the plan picks T and with T = 4 forced, then an
# alternating A/B of the learner legs against the previous commit's library (prev).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r6o && export TMPDIR=/tmp
O=$R/gpurun_out/r6o
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_learner_multi_gpu.py \
  tests/test_train_loop_gpu.py tests/test_dp_train_loop_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
MZ_MULTI_T=4 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_learner_multi_gpu.py \
  tests/test_train_loop_gpu.py > $O/tests4.log 2>&1 || { tail -30 $O/tests4.log; exit 1; }
tail -1 $O/tests4.log
for i in 1 2 3; do
  for v in ${VARIANTS:-prev cur}; do
    unset MZ_LIB
    [ $v != cur ] && export MZ_LIB=$R/muzero.jl_amd/lib/libmz_$v.so
    timeout -k 10 300 python bench.py --no-cpu --steps 5 --warmup 2 --pipeline-moves 0 --train-moves 10 > $O/ab_${v}_$i.log 2>&1 || { tail -20 $O/ab_${v}_$i.log; exit 1; }
    echo "$v $(tail -1 $O/ab_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('learner', d['learner_steps_per_s'], d['learner_multi']['call_ms'], d['learner_multi']['kernels'], 'train', round(d['train_loop']['node_expansions_per_s']/1e6,2))")"
  done
done
