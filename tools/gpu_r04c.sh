#!/bin/bash
# Tree-step phase stamps (prebuilt libmz_stamps.so) of the Atari-like and TicTacToe ResNet searches.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)} && mkdir -p gpurun_out/r4c
timeout -k 10 200 python tools/tree_stamps.py --no-build > gpurun_out/r4c/ts_atari.log 2>&1 || { tail -20 gpurun_out/r4c/ts_atari.log; exit 1; }
cat gpurun_out/r4c/ts_atari.log
GAME=ttt G=2048 timeout -k 10 200 python tools/tree_stamps.py --no-build > gpurun_out/r4c/ts_ttt.log 2>&1 || { tail -20 gpurun_out/r4c/ts_ttt.log; exit 1; }
cat gpurun_out/r4c/ts_ttt.log
