#!/bin/bash
# Per-variant ResNet network launch time (MZ_LIB, $LIBS; "base" = the in-tree libmz.so): the bench's
# roofline.kernel_ms (engine events on the launch stream) for configs[2].
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
for n in ${LIBS:-base}; do
  if [ "$n" = base ]; then unset MZ_LIB; else export MZ_LIB=$R/muzero.jl_amd/lib/libmz_$n.so; fi
  timeout -k 10 200 python bench.py --net resnet ${AB_ARGS} --no-cpu --steps 3 --warmup 1 --pipeline-moves 0 --train-moves 0 --learner-steps 5 > gpurun_out/abn_$n.log 2>&1 || { tail -20 gpurun_out/abn_$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/abn_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('exp/s', round(d['value']/1e6,2), 'nets_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])")"
done
