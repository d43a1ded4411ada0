#!/bin/bash
# ResNet (configs[2]) measurement: bench line + per-kernel rocprof stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python bench.py --net resnet ${BENCH_ARGS} > gpurun_out/rb.log 2>&1 || { tail -20 gpurun_out/rb.log; exit 1; }
tail -1 gpurun_out/rb.log
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/rprof" -o run -- \
      python "$R/bench.py" --net resnet --steps 5 --warmup 2 --learner-steps 20 --no-cpu > "$R/gpurun_out/rprof.log" 2>&1 \
      || { tail -20 "$R/gpurun_out/rprof.log"; exit 1; }
  f=$(find "$R/gpurun_out/rprof" -name "*kernel_stats.csv" | head -1)
  cut -d, -f1-8 "$f" | head -12
fi
