#!/bin/bash
# Round 5: the ResNet kernels with SLP vectorisation (packed f32 epilogue arithmetic) — ResNet / Atari
# parity, then alternating configs[2] / configs[4] search-only lines against HEAD's library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r5o && export TMPDIR=/tmp
O=$R/gpurun_out/r5o
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_resnet_gpu.py tests/test_atari_gpu.py tests/test_bench_sizes_gpu.py tests/test_learner_multi_gpu.py \
  tests/test_corrected_resnet_gpu.py tests/test_fault_gpu.py > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
b() {
  local n=$1; shift
  timeout -k 10 300 env "$@" > $O/$n.log 2>&1 || { echo "BENCH FAILED $n"; tail -20 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log | tail -1 > $O/$n.json
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
}
for rep in 1 2; do
  b rn_new_$rep python bench.py --no-cpu --search-only --net resnet
  b rn_head_$rep MZ_LIB=$R/muzero.jl_amd/lib/libmz_head.so python bench.py --no-cpu --search-only --net resnet
  b at_new_$rep python bench.py --no-cpu --search-only --game atari
  b at_head_$rep MZ_LIB=$R/muzero.jl_amd/lib/libmz_head.so python bench.py --no-cpu --search-only --game atari
done
