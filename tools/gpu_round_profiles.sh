#!/bin/bash
# Round profiles: kernel-trace stats of the default bench (configs[1]), FETCH_SIZE and WRITE_SIZE
# passes (separate runs) of the same command for the roofline traffic, and kernel-trace stats of
# the ResNet (configs[2]) and Atari-like (configs[4]) bench lines.  Usage: TAG=r01h bash tools/gpu_round_profiles.sh
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)} && mkdir -p gpurun_out/rp && export TMPDIR=/tmp
T=${TAG:-rXX}; O=gpurun_out/rp
B="python bench.py --steps 10 --warmup 2 --no-cpu --pipeline-moves 0 --learner-steps 50"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
# search-only dispatches (no self-play pipeline leg): the kernel's rocprof average is the bench's timed kernel_ms
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_search -o run -- python bench.py --pipeline-moves 0 > $O/bench_search.log 2>&1 || { tail -20 $O/bench_search.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > $O/fetch.log 2>&1 || { tail -20 $O/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $B > $O/write.log 2>&1 || { tail -20 $O/write.log; exit 1; }
python tools/pmc_summary.py $O/fetch $O/write mz_search_small2 $O/pmc_${T}_small2.json "$B" > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_resnet -o run -- python bench.py --net resnet --no-cpu > $O/bench_resnet.log 2>&1 || { tail -20 $O/bench_resnet.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_atari -o run -- python bench.py --game atari --no-cpu > $O/bench_atari.log 2>&1 || { tail -20 $O/bench_atari.log; exit 1; }
for f in default search resnet atari; do grep '^{' $O/bench_$f.log | tail -1 > $O/${T}_${f}_bench_under_rocprof.json; done
cp $O/kt/run_kernel_stats.csv $O/${T}_default_kernel_stats.csv
cp $O/kt_search/run_kernel_stats.csv $O/${T}_search_kernel_stats.csv
cp $O/kt_resnet/run_kernel_stats.csv $O/${T}_resnet_kernel_stats.csv
cp $O/kt_atari/run_kernel_stats.csv $O/${T}_atari_kernel_stats.csv
cat $O/pmc_${T}_small2.json; head -4 $O/${T}_default_kernel_stats.csv
