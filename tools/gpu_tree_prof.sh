set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lds -o run -- python bench.py --game atari --no-cpu --steps 3 --warmup 1 --pipeline-moves 0 > gpurun_out/p1.log 2>&1 || { tail -20 gpurun_out/p1.log; exit 1; }
MZ_RTREE_HBM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_hbm -o run -- python bench.py --game atari --no-cpu --steps 3 --warmup 1 --pipeline-moves 0 > gpurun_out/p2.log 2>&1 || { tail -20 gpurun_out/p2.log; exit 1; }
find gpurun_out/prof_lds gpurun_out/prof_hbm -name "*kernel_stats.csv" | xargs -I{} sh -c 'echo {}; head -8 {}'
