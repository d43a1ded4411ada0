#!/bin/bash
# Round 5: the ResNet / Atari tree step — recompute on the LDS pbc / sqrt tables and the path-only
# edge copy (second copy after a min / max move).  Parity (ResNet / Atari searches incl. the depth-199
# configs[4] launch), tree-step stamps, alternating A/B against MZ_RTREE_FULL_COPY=1, kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r5j && export TMPDIR=/tmp
O=$R/gpurun_out/r5j
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_atari_gpu.py tests/test_bench_sizes_gpu.py tests/test_resnet_gpu.py tests/test_fault_gpu.py \
  > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
MZ_RTREE_FULL_COPY=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_atari_gpu.py -k search > $O/tests_full.log 2>&1 || { echo "FULL-COPY TESTS FAILED"; tail -40 $O/tests_full.log; exit 1; }
tail -1 $O/tests_full.log
timeout -k 10 200 python tools/tree_stamps.py --no-build > $O/stamps.txt 2>&1 || { tail $O/stamps.txt; exit 1; }
b() {  # name, env..., -- args
  local n=$1; shift
  timeout -k 10 300 env "$@" > $O/$n.log 2>&1 || { echo "BENCH FAILED $n"; tail -20 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log | tail -1 > $O/$n.json
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['roofline']['kernel_ms'])"
}
for rep in 1 2; do
  b atari_po_$rep python bench.py --no-cpu --search-only --game atari
  b atari_full_$rep MZ_RTREE_FULL_COPY=1 python bench.py --no-cpu --search-only --game atari
done
b resnet_po python bench.py --no-cpu --search-only --net resnet
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python bench.py --no-cpu --search-only --game atari > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
head -6 $O/kt/run_kernel_stats.csv | cut -d, -f1-4


