#!/bin/bash
# A/B of prebuilt library variants (muzero.jl_amd/lib/libmz_<v>.so) on the default bench line
# (search kernel time and learner steps/s): VARIANTS="base v1" bash tools/ab_default.sh
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)} && mkdir -p gpurun_out
L=muzero.jl_amd/lib
cp $L/libmz.so $L/libmz_keep.so
for r in 1 2; do
for v in ${VARIANTS:-base}; do
  cp $L/libmz_$v.so $L/libmz.so
  timeout -k 10 300 python bench.py --no-cpu --pipeline-moves 0 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; cp $L/libmz_keep.so $L/libmz.so; exit 1; }
  echo $v $(grep '^{' gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'], d['learner_steps_per_s'])")
done
done
cp $L/libmz_keep.so $L/libmz.so
