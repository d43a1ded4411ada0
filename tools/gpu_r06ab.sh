#!/bin/bash
# Round 6 diagnostic: what bounds mz_learn_chain with one parameter per thread — this tree against the chain
# without ADAM's f64 arithmetic (-DMZ_DBG_CHEAP_ADAM) and without the bank scatter (-DMZ_DBG_NO_BANK); both
# diagnostics give wrong results (timing only).  Kernel-trace stats of the learner leg.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r6ab && export TMPDIR=/tmp
O=$R/gpurun_out/r6ab
B="--no-cpu --steps 2 --warmup 1 --pipeline-moves 0 --train-moves 0"
for v in cur xcheap xnobank; do
  if [ $v = cur ]; then unset MZ_LIB; else export MZ_LIB=$R/muzero.jl_amd/lib/libmz_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- python bench.py $B > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  echo "$v $(grep -E 'mz_learn_chain' $O/kt_$v/run_kernel_stats.csv | cut -d, -f1-4)"
done
