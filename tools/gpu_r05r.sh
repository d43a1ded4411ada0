#!/bin/bash
# Round 5 experiment: skew the middle wave of each SIMD at every ResNet layer (RN_SKEW sleep, variant
# libraries) against HEAD's library — configs[2] / configs[4] search-only lines, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r5r && export TMPDIR=/tmp
O=$R/gpurun_out/r5r
b() {
  local n=$1; shift
  timeout -k 10 300 env "$@" > $O/$n.log 2>&1 || { echo "BENCH FAILED $n"; tail -20 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log | tail -1 > $O/$n.json
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['roofline']['kernel_ms'])"
}
L=$R/muzero.jl_amd/lib
for rep in 1 2; do
  for v in head skew16 skew40; do
    b rn_${v}_$rep MZ_LIB=$L/libmz_$v.so python bench.py --no-cpu --search-only --net resnet
  done
  for v in head skew16 skew40; do
    b at_${v}_$rep MZ_LIB=$L/libmz_$v.so python bench.py --no-cpu --search-only --game atari
  done
done
