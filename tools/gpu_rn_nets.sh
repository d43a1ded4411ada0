#!/bin/bash
# ResNet search iteration: ResNet/Atari/Connect4 search parity subset, nets-kernel stamps
# (prebuilt libmz_stamps.so), the ResNet bench line.  Each step has its own limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_resnet_gpu.py tests/test_atari_gpu.py tests/test_bench_sizes_gpu.py \
    tests/test_selfplay_gpu.py -x -q --timeout 120 --timeout-method thread ${RN_K:+-k "$RN_K"} > gpurun_out/rt.log 2>&1 || { tail -30 gpurun_out/rt.log; exit 1; }
tail -1 gpurun_out/rt.log
timeout -k 10 120 python tools/rn_stamps.py --no-build > gpurun_out/nst.log 2>&1 || { tail -20 gpurun_out/nst.log; exit 1; }
grep -E "==|staging" gpurun_out/nst.log
timeout -k 10 200 python bench.py --net resnet --no-cpu --steps 5 --warmup 2 --pipeline-moves 0 --train-moves 0 --learner-steps 20 > gpurun_out/rb.log 2>&1 || { tail -20 gpurun_out/rb.log; exit 1; }
tail -1 gpurun_out/rb.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('exp/s', d['value'], 'nets_ms', d['roofline']['kernel_ms'], d['roofline']['frac'], 'learner', d['learner_steps_per_s'])"
