#!/bin/bash
# Round 6: which post-network phase is on the critical path — the search line with the expand's
# double softmax computed twice (x_exp2) and with the read-out activations twice (x_tanh2), same results.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r6i && export TMPDIR=/tmp
O=$R/gpurun_out/r6i
for i in 1 2; do
  for v in cur x_exp2 x_tanh2; do
    unset MZ_LIB
    [ $v != cur ] && export MZ_LIB=$R/muzero.jl_amd/lib/libmz_$v.so
    timeout -k 10 300 python bench.py --no-cpu --search-only --steps 20 --warmup 3 > $O/ab_${v}_$i.log 2>&1 || { tail -20 $O/ab_${v}_$i.log; exit 1; }
    echo "$v $(tail -1 $O/ab_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('exp/s', round(d['value']/1e6,2), d['roofline']['kernel_ms'])")"
  done
done
