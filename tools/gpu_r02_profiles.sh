#!/bin/bash
# Round-2 profiles (TAG=r02a ...): kernel-trace stats of the default (configs[1]), ResNet
# (configs[2]) and Atari-like (configs[4]) bench lines; per-kernel PMC of the search and
# learner kernels — FETCH_SIZE and WRITE_SIZE in separate passes (HBM traffic) and one SQ
# pass (VALU / MFMA instruction counts, busy and parked cycles) — summarised by
# tools/pmc_kernels.py.  Every GPU step has its own limit; the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/rp && export TMPDIR=/tmp
T=${TAG:-rXX}; O=$R/gpurun_out/rp
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES"
run() {  # name, limit, command...
  local n=$1 l=$2; shift 2
  timeout -k 10 $l "$@" > $O/$n.log 2>&1 || { echo "FAILED $n"; tail -20 $O/$n.log; exit 1; }
}
pmc() {  # tag, bench args, kernels...
  local t=$1 args=$2; shift 2
  run ${t}_fetch 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${t}_fetch -o run -- python bench.py $args
  run ${t}_write 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${t}_write -o run -- python bench.py $args
  run ${t}_sq 180 rocprofv3 --pmc $SQ --output-format csv -d $O/${t}_sq -o run -- python bench.py $args
  python tools/pmc_kernels.py $O/pmc2_${T}_${t}.json "python bench.py $args" $O/${t}_fetch $O/${t}_write $O/${t}_sq -- "$@" > /dev/null || exit 1
}
B1="--steps 10 --warmup 2 --no-cpu --pipeline-moves 0 --train-moves 0 --learner-steps 50"
if [ -z "$SKIP_DEFAULT" ]; then
run kt_default 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_default -o run -- python bench.py
pmc default "$B1" mz_search_small2 mz_learn_small1 mz_learn_multi2 mz_learn_chain mz_bp_tile_lv mz_bp_dw mz_bp_fold
fi
if [ -z "$SKIP_RESNET" ]; then
BR="--net resnet --steps 4 --warmup 1 --no-cpu --pipeline-moves 0 --train-moves 0 --learner-steps 10"
run kt_resnet 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_resnet -o run -- python bench.py --net resnet
pmc resnet "$BR" mz_rsearch_nets mz_runroll_fused_r mz_runroll_chain_r mz_runroll_pred_r mz_runroll_pred_n1 mz_rsearch_tree_lds mz_rsearch_root mz_learner_grad_kernel
fi
if [ -z "$SKIP_ATARI" ]; then
BA="--game atari --steps 2 --warmup 1 --no-cpu --learner-steps 10"
run kt_atari 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_atari -o run -- python bench.py --game atari
pmc atari "$BA" mz_rsearch_nets mz_runroll_chain mz_runroll_pred mz_rsearch_tree_lds32 mz_downsample_kernel
fi
for f in default resnet atari; do
  [ -f $O/kt_$f.log ] || continue
  grep '^{' $O/kt_$f.log | tail -1 > $O/${T}_${f}_bench_under_rocprof.json
  cp $O/kt_$f/run_kernel_stats.csv $O/${T}_${f}_kernel_stats.csv
done
ls $O
