#!/bin/bash
# ResNet iteration: learner/search parity subset, chain + nets stamps (prebuilt
# libmz_stamps.so), the ResNet bench line.  Each step has its own limit; the
# script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_resnet_gpu.py tests/test_atari_gpu.py tests/test_bench_sizes_gpu.py \
    tests/test_selfplay_gpu.py tests/test_checkpoint_gpu.py -x -q --timeout 120 --timeout-method thread \
    ${RN_K:+-k "$RN_K"} > gpurun_out/rt.log 2>&1 || { tail -30 gpurun_out/rt.log; exit 1; }
tail -1 gpurun_out/rt.log
timeout -k 10 120 python tools/rn_chain_stamps.py --no-build > gpurun_out/st_chain.log 2>&1 || { tail -20 gpurun_out/st_chain.log; exit 1; }
cat gpurun_out/st_chain.log
timeout -k 10 200 python bench.py --net resnet --no-cpu --steps 5 --warmup 2 --pipeline-moves 0 --train-moves 0 > gpurun_out/rb.log 2>&1 || { tail -20 gpurun_out/rb.log; exit 1; }
tail -1 gpurun_out/rb.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'nets_ms', d['roofline']['kernel_ms'], d['roofline']['frac'], 'learner', d['learner_steps_per_s'], d['learner_step_ms'], d['learner_roofline']['kernel_ms'])"
if [ -n "$RN_TRACE" ]; then
  export TMPDIR=/tmp
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rl -o run -- python bench.py --net resnet --no-cpu --steps 2 --warmup 1 --pipeline-moves 0 --train-moves 0 --learner-steps 100 > gpurun_out/rl.log 2>&1 || { tail -20 gpurun_out/rl.log; exit 1; }
  head -12 gpurun_out/rl/run_kernel_stats.csv | cut -d, -f1-4
fi
