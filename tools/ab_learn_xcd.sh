#!/bin/bash
# A/B of the FC learner's workgroup placement: the unroll workgroups on one XCD (MZ_LEARN_XCD=1)
# vs the plain grid (default), alternating bench runs; then the fused-learner parity tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_selfplay_gpu.py tests/test_fc_bn.py tests/test_train_loop_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "fused or prefetch or learner or train" > gpurun_out/lx_t.log 2>&1 || { tail -30 gpurun_out/lx_t.log; exit 1; }
tail -1 gpurun_out/lx_t.log
for i in 1 2 3; do
  for v in xcd plain; do
    if [ $v = xcd ]; then export MZ_LEARN_XCD=1; else unset MZ_LEARN_XCD; fi
    timeout -k 10 200 python bench.py --no-cpu --steps 3 --warmup 1 --pipeline-moves 0 --train-moves 0 --learner-steps 400 > gpurun_out/lx_$v.log 2>&1 || { tail -20 gpurun_out/lx_$v.log; exit 1; }
    echo "$v $(tail -1 gpurun_out/lx_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('learner', d['learner_steps_per_s'], d['learner_step_ms'])")"
  done
done
