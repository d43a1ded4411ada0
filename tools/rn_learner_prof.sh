#!/bin/bash
# ResNet learner unroll (split form): kernel-trace stats of a learner-only bench run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/rl && export TMPDIR=/tmp
B="python bench.py --net resnet --no-cpu --steps 2 --warmup 1 --pipeline-moves 0 --train-moves 0 --learner-steps 50"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rl/kt -o run -- $B > gpurun_out/rl/kt.log 2>&1 || { tail -20 gpurun_out/rl/kt.log; exit 1; }
head -8 gpurun_out/rl/kt/run_kernel_stats.csv
