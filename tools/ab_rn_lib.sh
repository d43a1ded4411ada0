#!/bin/bash
# A/B of prebuilt library variants on the configs[2] learner line (alternating runs):
# VARIANTS="base hs" bash tools/ab_rn_lib.sh   (libmz_<v>.so; base = the current libmz.so)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)} && mkdir -p gpurun_out
L=muzero.jl_amd/lib
cp $L/libmz.so $L/libmz_base.so
for r in 1 2; do
  for v in ${VARIANTS:-base}; do
    cp $L/libmz_$v.so $L/libmz.so
    timeout -k 10 300 python bench.py --net resnet --no-cpu --pipeline-moves 0 --steps 5 --learner-steps 300 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; cp $L/libmz_base.so $L/libmz.so; exit 1; }
    echo $v $(grep '^{' gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['learner_steps_per_s'])")
  done
done
cp $L/libmz_base.so $L/libmz.so
