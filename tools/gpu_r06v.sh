#!/bin/bash
# Round 6, the actor-learner loop's per-move overheads (trace of r6t: ~30-60 us from the count copies to the
# next launch, two ~4.5 us copy launches, four ~5 us actor repacks per move).  This tree: the count handed
# back by one kernel into coherent pinned memory and the host spinning on it; the chain launch writes the
# actors' search images itself.  A/B: MZ_TRAIN_SYNC=1 (copies + stream sync), MZ_TRAIN_REPACK=1 (repack).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r6v && export TMPDIR=/tmp
O=$R/gpurun_out/r6v
T="tests/test_learner_multi_gpu.py tests/test_train_loop_gpu.py tests/test_dp_train_loop_gpu.py tests/test_fault_gpu.py tests/test_selfplay_gpu.py"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $T > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B="--no-cpu --steps 3 --warmup 1 --pipeline-moves 0 --learner-steps 20 --train-moves 40"
for v in prev cur sync repack cur2; do
  if [ $v = prev ]; then export MZ_LIB=$R/muzero.jl_amd/lib/libmz_prev.so; else unset MZ_LIB; fi
  case $v in sync) export MZ_TRAIN_SYNC=1 ;; repack) unset MZ_TRAIN_SYNC; export MZ_TRAIN_REPACK=1 ;; *) unset MZ_TRAIN_SYNC MZ_TRAIN_REPACK ;; esac
  timeout -k 10 300 python bench.py $B > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  echo "$v $(grep '^{' $O/$v.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['train_loop']; print('train', t['node_expansions_per_s'], t['ms_per_move'], t['learner_steps'])")"
done
unset MZ_TRAIN_SYNC MZ_TRAIN_REPACK
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python bench.py $B > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
