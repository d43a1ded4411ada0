#!/bin/bash
# GPU tests, then an alternating A/B of the one-launch ResNet unroll (mz_runroll_fused_r)
# against the chain + prediction launches (MZ_RN_NO_FUSE=1) on the ResNet learner lines.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)} && mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for r in 1 2; do
  for v in ${AB_VARIANTS:-fuse nofuse}; do
    for a in "--net resnet"; do
      E="MZ_AB=$v"; [ $v = nofuse ] && E="MZ_RN_NO_FUSE=1"; [ $v = nofs ] && E="MZ_RN_NO_FUSE_SAMPLE=1"
      env $E timeout -k 10 300 python bench.py $a --no-cpu --pipeline-moves 0 --steps 5 --learner-steps 200 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
      echo $v $a $(grep '^{' gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['learner_steps_per_s'], d.get('learner_roofline',{}).get('kernel'))")
    done
  done
done
