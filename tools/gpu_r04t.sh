#!/bin/bash
# Corrected-learner tests on HEAD's libmz, then an alternating A/B of the FC
# corrected leg (libmz vs libmz_old, the previous build).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r4t && export TMPDIR=/tmp
O=$R/gpurun_out/r4t
timeout -k 10 400 python -u -m pytest tests/test_corrected_learner_gpu.py tests/test_fc_bn.py tests/test_dp_libmz_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
v() { grep '^{' $1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['learner_corrected']; print(c['learner_steps_per_s'], c['step_ms'])"; }
for i in 1 2 3; do
  for n in base old; do
    if [ $n = base ]; then unset MZ_LIB; else export MZ_LIB=$R/muzero.jl_amd/lib/libmz_$n.so; fi
    timeout -k 10 300 python bench.py --no-cpu --steps 4 --warmup 1 --pipeline-moves 0 --train-moves 0 --learner-steps 100 > $O/c_${n}_$i.log 2>&1 || { tail -20 $O/c_${n}_$i.log; exit 1; }
    echo "corrected $n $i $(v $O/c_${n}_$i.log)"
  done
done
