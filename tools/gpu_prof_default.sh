#!/bin/bash
# rocprofv3 kernel-trace summary of the default bench line (configs[1]).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)} && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_default -o run -- python bench.py ${BENCH_ARGS} > gpurun_out/prof_default.log 2>&1 || { tail -20 gpurun_out/prof_default.log; exit 1; }
grep '^{' gpurun_out/prof_default.log | tail -1 | cut -c1-300
head -14 gpurun_out/prof_default/run_kernel_stats.csv
