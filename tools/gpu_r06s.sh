#!/bin/bash
# Round 6 diagnostic: the FC chain launch with each thread's first parameter only (-DMZ_DBG_ONE_ELEM, wrong
# results, timing only) against this tree.  At 128 slices x 256 threads per net, the prediction net's 33,308
# parameters give 540 threads a second parameter; if the chain is bound by the slowest thread's serial
# 2 x 32 ADAM iterations, the one-parameter chain runs in about half the time.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r6s && export TMPDIR=/tmp
O=$R/gpurun_out/r6s
for v in prev xone; do
  export MZ_LIB=$R/muzero.jl_amd/lib/libmz_$v.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- python bench.py --no-cpu --steps 3 --warmup 1 --pipeline-moves 0 --train-moves 0 > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  echo "$v $(grep '^{' $O/$v.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('learner', d['learner_steps_per_s'], d['learner_multi']['call_ms'])")"
  grep -E "mz_learn_chain|mz_learn_multi" $O/kt_$v/run_kernel_stats.csv | cut -d, -f1-4
done
