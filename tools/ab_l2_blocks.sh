#!/bin/bash
# Σθ² / ADAM slice count A/B (timing only; libmz_l2_<n>.so built with -DMZ_L2_BLOCKS=n):
# the ResNet learner's kernel trace and the FC learner rate per variant.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/l2 && export TMPDIR=/tmp
L=muzero.jl_amd/lib
cp $L/libmz.so $L/libmz_base.so
B="python bench.py --net resnet --no-cpu --steps 2 --warmup 1 --pipeline-moves 0 --train-moves 0 --learner-steps 200"
for v in ${VARIANTS:-base l2_32 l2_512}; do
  cp $L/libmz_$v.so $L/libmz.so
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/l2/$v -o run -- $B > gpurun_out/l2/$v.log 2>&1 || { tail -20 gpurun_out/l2/$v.log; exit 1; }
  echo "== $v"; python tools/trace_gaps.py gpurun_out/l2/$v/run_kernel_trace.csv runroll learner_grad
  timeout -k 10 300 python bench.py --no-cpu --pipeline-moves 0 --train-moves 0 --steps 5 > gpurun_out/l2/fc_$v.log 2>&1 || { tail -20 gpurun_out/l2/fc_$v.log; exit 1; }
  echo $v FC learner $(grep '^{' gpurun_out/l2/fc_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['learner_steps_per_s'])")
done
cp $L/libmz_base.so $L/libmz.so
