#!/bin/bash
# A/B of prebuilt library variants (muzero.jl_amd/lib/libmz_<v>.so, built here with
# different -D flags) on the ResNet and Atari bench lines: VARIANTS="base v1 v2" bash tools/ab_resnet.sh
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=muzero.jl_amd/lib
cp $L/libmz.so $L/libmz_keep.so
for v in ${VARIANTS:-base}; do
  cp $L/libmz_$v.so $L/libmz.so
  for a in "--net resnet" "--game atari"; do
    timeout -k 10 300 python bench.py $a --no-cpu --pipeline-moves 0 --steps 10 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    echo $v $a $(grep '^{' gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'], d['learner_steps_per_s'])")
  done
done
cp $L/libmz_keep.so $L/libmz.so
