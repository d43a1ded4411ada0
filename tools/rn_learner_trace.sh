#!/bin/bash
# ResNet learner (configs[2] learner leg): kernel traces of the one-launch unroll and of
# the chain + prediction launches (MZ_RN_NO_FUSE=1), and without the fused ADAM blocks
# (MZ_RN_NO_FUSE_ADAM=1); per-kernel durations and launch gaps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/rl && export TMPDIR=/tmp
B="python bench.py --net resnet --no-cpu --steps 2 --warmup 1 --pipeline-moves 0 --train-moves 0 --learner-steps 200"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rl/fuse -o run -- $B > gpurun_out/rl/fuse.log 2>&1 || { tail -20 gpurun_out/rl/fuse.log; exit 1; }
MZ_RN_NO_FUSE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rl/nofuse -o run -- $B > gpurun_out/rl/nofuse.log 2>&1 || { tail -20 gpurun_out/rl/nofuse.log; exit 1; }
MZ_RN_NO_FUSE_ADAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rl/noadam -o run -- $B > gpurun_out/rl/noadam.log 2>&1 || { tail -20 gpurun_out/rl/noadam.log; exit 1; }
for v in fuse noadam nofuse; do echo "== $v"; python tools/trace_gaps.py gpurun_out/rl/$v/run_kernel_trace.csv runroll rp_sample learner_grad; done
