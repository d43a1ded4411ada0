#!/bin/bash
# A/B of library variants (MZ_LIB) on the ResNet bench line: learner steps/s and the
# search network launch, per lib in $LIBS (names under muzero.jl_amd/lib/libmz_<name>.so;
# "base" = the in-tree libmz.so).  Each run has its own limit; stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
for n in ${LIBS:-base}; do
  if [ "$n" = base ]; then unset MZ_LIB; else export MZ_LIB=$R/muzero.jl_amd/lib/libmz_$n.so; fi
  timeout -k 10 200 python bench.py --net resnet ${AB_ARGS} --no-cpu --steps 3 --warmup 1 --pipeline-moves 0 --train-moves 0 --learner-steps 100 > gpurun_out/ab_$n.log 2>&1 || { tail -20 gpurun_out/ab_$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/ab_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('exp/s', round(d['value']/1e6,2), 'nets_ms', d['roofline']['kernel_ms'], 'learner', d['learner_steps_per_s'], d['learner_step_ms'])")"
done
