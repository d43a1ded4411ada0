#!/bin/bash
# Alternating A/B/C of the configs[4] search-only line: libmz (4 recompute rows per group and pass in the
# tree step) vs libmz_u2 (-DRT_RECOMP_U=2) vs libmz_u6 (-DRT_RECOMP_U=6), the Atari parity subset on both first.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r5u && export TMPDIR=/tmp
O=$R/gpurun_out/r5u
for n in u2 u6; do
  MZ_LIB=$R/muzero.jl_amd/lib/libmz_$n.so timeout -k 10 400 python -u -m pytest tests/test_atari_gpu.py tests/test_bench_launch_gpu.py tests/test_bench_sizes_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "atari or configs4 or depth" > $O/t_$n.log 2>&1 || { tail -30 $O/t_$n.log; exit 1; }
  echo "$n $(tail -n 1 $O/t_$n.log)"
done
v() { grep '^{' $1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,3))"; }
for i in 1 2 3; do
  for n in base u2 u6; do
    if [ $n = base ]; then unset MZ_LIB; else export MZ_LIB=$R/muzero.jl_amd/lib/libmz_$n.so; fi
    timeout -k 10 300 python bench.py --game atari --no-cpu --search-only --steps 3 --warmup 1 > $O/a_${n}_$i.log 2>&1 || { tail -20 $O/a_${n}_$i.log; exit 1; }
    echo "atari $n $i $(v $O/a_${n}_$i.log)"
  done
done
