#!/bin/bash
# Round 5: the chain launch's duration by chunk length, with and without the bank scatter
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r5c && export TMPDIR=/tmp
O=$R/gpurun_out/r5c
for v in base nobank; do
  [ $v = nobank ] && export MZ_LIB=$R/muzero.jl_amd/lib/libmz_nobank.so
  for L in 1 4 8 16; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}_$L -o run -- python tools/chain_probe.py $L > $O/${v}_$L.log 2>&1 || { tail -5 $O/${v}_$L.log; exit 1; }
    echo "$v L=$L $(grep -h 'mz_learn_chain\|mz_learn_multi' $O/${v}_$L/run_kernel_stats.csv | cut -d, -f1,2,4 | tr '\n' ' ')"
  done
done
