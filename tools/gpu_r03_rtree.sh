#!/bin/bash
# Round-3 iteration: ResNet / Atari parity with the cached select in the LDS tree step, the tree
# step's phase stamps (Atari-like, TicTacToe ResNet), ResNet and Atari bench lines.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)} && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_resnet_gpu.py tests/test_atari_gpu.py tests/test_bench_launch_gpu.py tests/test_train_loop_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/rt.log 2>&1 || { tail -30 gpurun_out/rt.log; exit 1; }
tail -2 gpurun_out/rt.log
timeout -k 10 200 python tools/tree_stamps.py --no-build > gpurun_out/ts_atari.log 2>&1 && tail -12 gpurun_out/ts_atari.log || exit 1
GAME=ttt timeout -k 10 200 python tools/tree_stamps.py --no-build > gpurun_out/ts_ttt.log 2>&1 && tail -6 gpurun_out/ts_ttt.log || exit 1
timeout -k 10 300 python bench.py --net resnet --no-cpu > gpurun_out/b_resnet.log 2>&1 && tail -1 gpurun_out/b_resnet.log | cut -c1-300 || exit 1
timeout -k 10 300 python bench.py --game atari --no-cpu > gpurun_out/b_atari.log 2>&1 && tail -1 gpurun_out/b_atari.log | cut -c1-300
