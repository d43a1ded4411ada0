#!/bin/bash
# A/B of library variants (MZ_LIB) on the default bench line (configs[1]): FC parity subset on
# the variant ($PARITY_K), then the bench per lib in $LIBS ("base" = the in-tree libmz.so).
# Each run has its own limit; stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
if [ -n "$PARITY_LIB" ]; then
  MZ_LIB=$R/muzero.jl_amd/lib/libmz_$PARITY_LIB.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py \
      tests/test_bench_sizes_gpu.py tests/test_selfplay_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
      -k "${PARITY_K:-small or dispatch or golden or games or configs1 or fused}" > gpurun_out/ab_t.log 2>&1 || { tail -30 gpurun_out/ab_t.log; exit 1; }
  tail -1 gpurun_out/ab_t.log
fi
for n in ${LIBS:-base}; do
  if [ "$n" = base ]; then unset MZ_LIB; else export MZ_LIB=$R/muzero.jl_amd/lib/libmz_$n.so; fi
  timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 3 --pipeline-moves 10 --train-moves 0 ${AB_ARGS} > gpurun_out/abd_$n.log 2>&1 || { tail -20 gpurun_out/abd_$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/abd_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('exp/s', round(d['value']/1e6,2), d['roofline']['kernel'], d['roofline']['kernel_ms'], 'learner', d['learner_steps_per_s'], 'pipe', round(d['selfplay_pipeline']['node_expansions_per_s']/1e6,2))")"
done
