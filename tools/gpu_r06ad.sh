#!/bin/bash
# Round 6: the ResNet search without the per-simulation copy of the parent's h — the tree step counts the
# parent's in-place doublings (Q1) and the network launch reads hid[leaf] times 2^k (exact).  Model: the
# gather moved 3·H floats per game per simulation (configs[2]: 14 MB per tree step).  The whole GPU suite,
# then search-only lines of configs[2]-[4] against HEAD (prev), alternating, and kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r6ad && export TMPDIR=/tmp
O=$R/gpurun_out/r6ad
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in "config2 --net resnet" "config3 --game connect4 --net resnet" "config4 --game atari --steps 3"; do
  set -- $c; n=$1; shift
  for v in prev cur prev2 cur2; do
    if [ ${v%2} = prev ]; then export MZ_LIB=$R/muzero.jl_amd/lib/libmz_prev.so; else unset MZ_LIB; fi
    timeout -k 10 300 python bench.py --search-only --no-cpu "$@" > $O/${n}_$v.log 2>&1 || { tail -20 $O/${n}_$v.log; exit 1; }
    echo "$n $v $(grep '^{' $O/${n}_$v.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])")"
  done
done
unset MZ_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_rn -o run -- python bench.py --search-only --no-cpu --net resnet > $O/kt_rn.log 2>&1 || { tail -20 $O/kt_rn.log; exit 1; }
grep -E "mz_rsearch" $O/kt_rn/run_kernel_stats.csv | cut -d, -f1-4
