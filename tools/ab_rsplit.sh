#!/bin/bash
# GPU tests, then an alternating A/B of the reward-head split of mz_rsearch_nets
# (default) against the prediction / dynamics split (MZ_RN_NO_RSPLIT=1) on configs[2], [3], [4].
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)} && mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for r in 1 2; do
  for v in split nosplit; do
    for a in "--net resnet" "--game connect4 --net resnet" "--game atari"; do
      E="MZ_AB=$v"; [ $v = nosplit ] && E="MZ_RN_NO_RSPLIT=1"
      env $E timeout -k 10 300 python bench.py $a --no-cpu --pipeline-moves 0 --train-moves 0 --steps 8 --learner-steps 20 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
      echo $v $a $(grep '^{' gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], r['kernel'], r['kernel_ms'], r['frac'])")
    done
  done
done
