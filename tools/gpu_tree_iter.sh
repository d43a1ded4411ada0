#!/bin/bash
# Tree-step iteration: ResNet/Atari GPU parity, tree stamps, Atari + ResNet bench lines.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)} && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_atari_gpu.py tests/test_resnet_gpu.py tests/test_selfplay_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 200 python tools/tree_stamps.py --no-build > gpurun_out/ts.log 2>&1 || { tail -20 gpurun_out/ts.log; exit 1; }
sed -n '1p;8,12p;27,30p' gpurun_out/ts.log
timeout -k 10 300 python bench.py --game atari --no-cpu > gpurun_out/bench_atari.log 2>&1 || { tail -20 gpurun_out/bench_atari.log; exit 1; }
tail -1 gpurun_out/bench_atari.log | cut -c1-200
timeout -k 10 300 python bench.py --net resnet --no-cpu --pipeline-moves 0 > gpurun_out/bench_resnet.log 2>&1 || { tail -20 gpurun_out/bench_resnet.log; exit 1; }
tail -1 gpurun_out/bench_resnet.log | cut -c1-200
