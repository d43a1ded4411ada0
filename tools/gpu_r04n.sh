#!/bin/bash
# The -m gpu suite with the skip-ahead after a min / max move (FC and ResNet tree
# steps), then alternating A/B: configs[1] (libmz vs libmz_nms, built with
# -DMZ_NO_MOVED_SKIP) and configs[4] (MZ_NO_MOVED_SKIP=1 vs not) search-only lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r4n && export TMPDIR=/tmp
O=$R/gpurun_out/r4n
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
fi
v() { grep '^{' $1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,3), d['roofline']['kernel'], d['roofline']['kernel_ms'])"; }
for i in 1 2; do
  for n in base nms; do
    if [ $n = base ]; then unset MZ_LIB; else export MZ_LIB=$R/muzero.jl_amd/lib/libmz_nms.so; fi
    timeout -k 10 200 python bench.py --no-cpu --search-only --steps 20 --warmup 3 > $O/d_${n}_$i.log 2>&1 || { tail -20 $O/d_${n}_$i.log; exit 1; }
    echo "default $n $i $(v $O/d_${n}_$i.log)"
  done
done
unset MZ_LIB
for i in 1 2; do
  for n in base nms; do
    if [ $n = base ]; then unset MZ_NO_MOVED_SKIP; else export MZ_NO_MOVED_SKIP=1; fi
    timeout -k 10 300 python bench.py --game atari --no-cpu --search-only --steps 3 --warmup 1 > $O/a_${n}_$i.log 2>&1 || { tail -20 $O/a_${n}_$i.log; exit 1; }
    echo "atari $n $i $(v $O/a_${n}_$i.log)"
  done
done
