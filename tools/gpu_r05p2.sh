#!/bin/bash
# Alternating A/B of the configs[4] search-only line: libmz vs libmz_pre (-DMZ_BK1P_PRE:
# the one-player backup update loop reads four of its levels per lane before any store),
# parity subset on the variant first.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r5p2 && export TMPDIR=/tmp
O=$R/gpurun_out/r5p2
MZ_LIB=$R/muzero.jl_amd/lib/libmz_pre.so timeout -k 10 400 python -u -m pytest tests/test_atari_gpu.py tests/test_bench_launch_gpu.py tests/test_bench_sizes_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "atari or configs4 or depth" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
v() { grep '^{' $1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,3))"; }
for i in 1 2 3; do
  for n in base pre; do
    if [ $n = base ]; then unset MZ_LIB; else export MZ_LIB=$R/muzero.jl_amd/lib/libmz_$n.so; fi
    timeout -k 10 300 python bench.py --game atari --no-cpu --search-only --steps 3 --warmup 1 > $O/a_${n}_$i.log 2>&1 || { tail -20 $O/a_${n}_$i.log; exit 1; }
    echo "atari $n $i $(v $O/a_${n}_$i.log)"
  done
done
