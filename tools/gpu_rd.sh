#!/bin/bash
# ResNet learner iteration: learner parity subset, then the ResNet bench line with and without
# the resident dynamics chain (MZ_RN_NO_RD=1).  Each step has its own limit; stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_resnet_gpu.py tests/test_atari_gpu.py tests/test_bench_sizes_gpu.py \
    tests/test_selfplay_gpu.py tests/test_checkpoint_gpu.py tests/test_train_loop_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "${RN_K:-learner or fused or configs3 or resume or train}" > gpurun_out/rt.log 2>&1 || { tail -30 gpurun_out/rt.log; exit 1; }
tail -1 gpurun_out/rt.log
for v in new old new old; do
  if [ $v = old ]; then export MZ_RN_NO_RD=1; else unset MZ_RN_NO_RD; fi
  timeout -k 10 200 python bench.py --net resnet ${AB_ARGS} --no-cpu --steps 3 --warmup 1 --pipeline-moves 0 --train-moves 0 --learner-steps 100 > gpurun_out/rd_$v.log 2>&1 || { tail -20 gpurun_out/rd_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/rd_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('learner', d['learner_steps_per_s'], d['learner_step_ms'], d['learner_roofline']['kernel_ms'])")"
done
