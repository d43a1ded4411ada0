#!/bin/bash
# ResNet corrected learner A/B (rbp_conv_dt loads batched): its torch-f64 tests, then base / head alternated
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r05w
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_corrected_resnet_gpu.py tests/test_dp_libmz_gpu.py > gpurun_out/r05w/tests.log 2>&1 || { tail -30 gpurun_out/r05w/tests.log; exit 1; }
tail -2 gpurun_out/r05w/tests.log
LIBS="${LIBS:-base head base head}" bash tools/ab_rbp.sh
