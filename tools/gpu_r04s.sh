#!/bin/bash
# FC learner / loss-term parity subset on HEAD's libmz, then an alternating A/B of
# the configs[1] learner (libmz vs libmz_old, the previous build).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r4s && export TMPDIR=/tmp
O=$R/gpurun_out/r4s
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_selfplay_gpu.py tests/test_train_loop_gpu.py tests/test_fc_bn.py tests/test_bench_sizes_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
v() { grep '^{' $1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,3), d['learner_steps_per_s'], d['learner_roofline'].get('kernel_ms'))"; }
for i in 1 2 3; do
  for n in base old; do
    if [ $n = base ]; then unset MZ_LIB; else export MZ_LIB=$R/muzero.jl_amd/lib/libmz_$n.so; fi
    timeout -k 10 300 python bench.py --no-cpu --steps 10 --warmup 2 --pipeline-moves 0 --train-moves 0 --learner-steps 400 > $O/d_${n}_$i.log 2>&1 || { tail -20 $O/d_${n}_$i.log; exit 1; }
    echo "default $n $i $(v $O/d_${n}_$i.log)"
  done
done
