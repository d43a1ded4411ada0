#!/bin/bash
# Instruction / scalar cache counters of the ResNet kernels (one PMC pass).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/ic && export TMPDIR=/tmp
B="python bench.py --net resnet --no-cpu --steps 2 --warmup 1 --pipeline-moves 0 --train-moves 0 --learner-steps 20"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM --output-format csv -d gpurun_out/ic/p1 -o run -- $B > gpurun_out/ic/p1.log 2>&1 || { tail -20 gpurun_out/ic/p1.log; exit 1; }
python tools/pmc_kernels.py gpurun_out/ic/ic.json "$B" gpurun_out/ic/p1 -- mz_runroll_chain mz_runroll_pred mz_rsearch_nets mz_rsearch_tree_lds > /dev/null && cat gpurun_out/ic/ic.json
