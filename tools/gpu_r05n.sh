#!/bin/bash
# Round 5: the downsampler's BatchNorm quotient by the exact reciprocal form — Atari parity
# (forward, search incl. the configs[4] launch, learners one-step / multi-step / corrected),
# per-layer stamps at 32 and 512 items, and the kernel's rocprof average in the configs[4] line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r5n && export TMPDIR=/tmp
O=$R/gpurun_out/r5n
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_atari_gpu.py tests/test_bench_sizes_gpu.py tests/test_learner_multi_gpu.py tests/test_corrected_resnet_gpu.py \
  > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for n in 32 512; do
  MZ_LIB=$R/muzero.jl_amd/lib/libmz_stamps.so timeout -k 10 120 python tools/ds_stamps.py $n > $O/ds$n.txt 2>&1 || { tail $O/ds$n.txt; exit 1; }
  grep total $O/ds$n.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python bench.py --no-cpu --game atari > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
grep -h "mz_downsample_kernel\|mz_rsearch_nets\"\|mz_rsearch_tree_lds32" $O/kt/run_kernel_stats.csv | cut -d, -f1-4
grep '^{' $O/prof.log | tail -1 > $O/atari_prof_line.json
