#!/bin/bash
# Round 6: the cached select walk with the next level's entry read before this level's path bookkeeping
# (stamps: 7.24 levels x 275 ticks per simulation, the LDS latency exposed each level; model: ~60-80 of the
# 275 hidden, ~3 % of the configs[1] launch).  The whole GPU suite, then search-only lines against HEAD (prev),
# alternating: configs[1], configs[2] and configs[4] (the ResNet tree step walks the same way).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r6ag && export TMPDIR=/tmp
O=$R/gpurun_out/r6ag
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in "config1 --steps 20" "config2 --net resnet" "config4 --game atari --steps 3"; do
  set -- $c; n=$1; shift
  for v in prev cur prev2 cur2; do
    if [ ${v%2} = prev ]; then export MZ_LIB=$R/muzero.jl_amd/lib/libmz_prev.so; else unset MZ_LIB; fi
    timeout -k 10 300 python bench.py --search-only --no-cpu "$@" > $O/${n}_$v.log 2>&1 || { tail -20 $O/${n}_$v.log; exit 1; }
    echo "$n $v $(grep '^{' $O/${n}_$v.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])")"
  done
done
