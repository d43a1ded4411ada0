#!/bin/bash
# Round-6 default-line pass (T = r06zh, after the pipelined select walk): configs[1] and [0], the search and default kernel stats, PMC default; one clean bench line per BASELINE config (no profiler),
# the search-only default command under kernel-trace stats, then per line
# (default / resnet / atari) FETCH_SIZE, WRITE_SIZE and one SQ pass, each its own
# rocprofv3 run, folded by tools/pmc_kernels.py.  Each GPU step has its own limit;
# the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r6zh && export TMPDIR=/tmp
O=$R/gpurun_out/r6zh; T=r06zh
if [ -z "$SKIP_CONFIGS" ]; then
run() {  # name, limit, bench args...
  local n=$1 l=$2; shift 2
  timeout -k 10 $l python bench.py "$@" > $O/$n.log 2>&1 || { echo "FAILED $n"; tail -20 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log | tail -1 > $O/${T}_${n}_bench.json
  python -c "import json,sys; d=json.load(open('$O/${T}_${n}_bench.json')); c=d.get('learner_corrected') or {}; print('$n', d['value'], d.get('learner_steps_per_s'), d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'), 'corrected', c.get('learner_steps_per_s'))"
}
run config1 300
run config0 200 --games 1 --sims 25 --learner-steps 50 --train-moves 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_search -o run -- python bench.py --search-only --no-cpu > $O/search.log 2>&1 || { tail -20 $O/search.log; exit 1; }
cp $O/kt_search/run_kernel_stats.csv $O/${T}_search_kernel_stats.csv
head -4 $O/${T}_search_kernel_stats.csv | cut -d, -f1-4
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_default -o run -- python bench.py --no-cpu > $O/default_prof.log 2>&1 || { tail -20 $O/default_prof.log; exit 1; }
cp $O/kt_default/run_kernel_stats.csv $O/${T}_default_kernel_stats.csv
grep '^{' $O/default_prof.log | tail -1 > $O/${T}_default_bench_under_rocprof.json
head -8 $O/${T}_default_kernel_stats.csv | cut -d, -f1-4
fi
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES"
for line in ${LINES:-default}; do
  case $line in
    default) A=""; K="mz_search_small2 mz_learn_small1 mz_learn_multi4 mz_learn_multi1 mz_learn_multi2 mz_learn_chain mz_bp_tile_lv_nobn mz_bp_dw mz_bp_fold";;
    resnet) A="--net resnet"; K="mz_rsearch_nets mz_rsearch_tree_lds mz_rsearch_root mz_runroll_fused_r mz_learn_chain mz_learner_loss_multi mz_rbp_sample mz_rbp_dw";;
    atari) A="--game atari"; K="mz_rsearch_nets mz_rsearch_tree_lds32 mz_rsearch_root32 mz_downsample_kernel mz_runroll_chain1 mz_runroll_pred_n1 mz_learn_chain mz_learner_loss_multi mz_dsbp_fwd mz_dsbp_bwd mz_dsbp_dw mz_rbp_sample";;
  esac
  B="python bench.py $A --steps 4 --warmup 1 --no-cpu --pipeline-moves 0 --train-moves 0 --learner-steps 10"
  dirs=""
  for c in FETCH_SIZE WRITE_SIZE SQ; do
    ctr=$c; [ $c = SQ ] && ctr="$SQ"
    timeout -s KILL 200 rocprofv3 --pmc $ctr --output-format csv -d $O/${line}_$c -o run -- $B > $O/${line}_$c.log 2>&1 || { echo "FAILED $line $c"; tail -5 $O/${line}_$c.log; exit 1; }
    dirs="$dirs $O/${line}_$c"
  done
  python tools/pmc_kernels.py $O/pmc2_${T}_${line}.json "$B" $dirs -- $K > /dev/null
  python -c "import json; d=json.load(open('$O/pmc2_${T}_${line}.json')); print('$line', {k: (round(v.get('hbm_bytes_per_launch_fetch_x2', 0)), round(v.get('wait_any_frac', 0), 3), round(v.get('mfma_util_chip', 0), 4)) for k, v in d['kernels'].items()})"
done
