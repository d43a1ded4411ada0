#!/bin/bash
# Atari parity subset on HEAD's libmz, then an alternating A/B of the configs[4]
# line (search-only value and the learner, whose batches run the downsampler):
# libmz (HEAD) vs libmz_new (the variant under test, parity-checked first).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r4u && export TMPDIR=/tmp
O=$R/gpurun_out/r4u
MZ_LIB=$R/muzero.jl_amd/lib/libmz_new.so timeout -k 10 500 python -u -m pytest tests/test_atari_gpu.py tests/test_atari_env.py tests/test_bench_launch_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
v() { grep '^{' $1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,3), d['learner_steps_per_s'])"; }
for i in 1 2 3; do
  for n in base new; do
    if [ $n = base ]; then unset MZ_LIB; else export MZ_LIB=$R/muzero.jl_amd/lib/libmz_$n.so; fi
    timeout -k 10 300 python bench.py --game atari --no-cpu --steps 3 --warmup 1 --pipeline-moves 0 --train-moves 0 --learner-steps 40 > $O/a_${n}_$i.log 2>&1 || { tail -20 $O/a_${n}_$i.log; exit 1; }
    echo "atari $n $i $(v $O/a_${n}_$i.log)"
  done
done
