#!/bin/bash
# Round 5: (1) the FC corrected learner with the BatchNorm test compiled out
# (mz_bp_tile_lv_nobn) against HEAD's library, alternating; (2) the N > 1 bench
# path with 8 gloo ranks on this one GPU (replica checks after the learner legs).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r5d && export TMPDIR=/tmp
O=$R/gpurun_out/r5d
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_corrected_learner_gpu.py tests/test_fc_bn.py > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
b() {  # name, lib
  local n=$1 lib=$2
  MZ_LIB=$lib timeout -k 10 200 python bench.py --no-cpu --pipeline-moves 0 --steps 5 --train-moves 0 --learner-chunk 1 > $O/$n.log 2>&1 || { echo "FAILED $n"; tail -5 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log | tail -1 > $O/$n.json
  python -c "import json; d=json.load(open('$O/$n.json')); c=d['learner_corrected']; print('$n', c['learner_steps_per_s'], c['step_ms'])"
}
for rep in 1 2; do
  b new_$rep $R/muzero.jl_amd/lib/libmz.so
  b head_$rep $R/muzero.jl_amd/lib/libmz_head.so
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python bench.py --no-cpu --pipeline-moves 0 --steps 5 --train-moves 0 --learner-chunk 1 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
grep -h "mz_bp_" $O/kt/run_kernel_stats.csv | cut -d, -f1-4
MZ_DIST_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 8 --game connect4 --net resnet --steps 5 --warmup 2 --learner-steps 20 > $O/gloo8.log 2>&1 || { echo "FAILED gloo8"; tail -20 $O/gloo8.log; exit 1; }
grep '^{' $O/gloo8.log | tail -1 > $O/r05d_gloo8_connect4_resnet_bench.json
python -c "import json; d=json.load(open('$O/r05d_gloo8_connect4_resnet_bench.json')); print('gloo8', d['n_gpus'], d['value'], d['learner_steps_per_s'], d['replica_checks'], d['learner_corrected']['learner_steps_per_s'])"
