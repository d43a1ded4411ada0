#!/bin/bash
# Round 6: the chain helpers on by default (FC and ResNet nets).  Parity: the learner / train-loop / ResNet /
# Atari / fault tests; then the learner rates of configs[2]-[4] for HEAD (prev) and this tree (no profiler).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r6u && export TMPDIR=/tmp
O=$R/gpurun_out/r6u
T="tests/test_learner_multi_gpu.py tests/test_train_loop_gpu.py tests/test_dp_train_loop_gpu.py tests/test_fault_gpu.py tests/test_resnet_gpu.py tests/test_atari_gpu.py"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $T > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for c in "config2 --net resnet" "config3 --game connect4 --net resnet" "config4 --game atari"; do
  set -- $c; n=$1; shift
  for v in prev cur; do
    if [ $v = cur ]; then unset MZ_LIB; else export MZ_LIB=$R/muzero.jl_amd/lib/libmz_$v.so; fi
    timeout -k 10 400 python bench.py --no-cpu --pipeline-moves 0 "$@" > $O/${n}_$v.log 2>&1 || { tail -20 $O/${n}_$v.log; exit 1; }
    echo "$n $v $(grep '^{' $O/${n}_$v.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'learner', d['learner_steps_per_s'], 'train', (d.get('train_loop') or {}).get('node_expansions_per_s'))")"
  done
done
