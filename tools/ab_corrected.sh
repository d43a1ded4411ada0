#!/bin/bash
# A/B of library variants (MZ_LIB) on the corrected learner leg (FC, B = 32, K = 5), per lib in $LIBS
# ("base" = the in-tree libmz.so).  Each run has its own limit; stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
for n in ${LIBS:-base}; do
  if [ "$n" = base ]; then unset MZ_LIB; else export MZ_LIB=$R/muzero.jl_amd/lib/libmz_$n.so; fi
  timeout -k 10 200 python bench.py --no-cpu --steps 2 --warmup 1 --pipeline-moves 0 --train-moves 0 --learner-steps 40 ${AB_ARGS} > gpurun_out/abc_$n.log 2>&1 || { tail -20 gpurun_out/abc_$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/abc_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['learner_corrected']; print(c['learner_steps_per_s'], c['step_ms'])")"
done
