#!/bin/bash
# Round 6: the backup's loads issued before the read-outs (backup_preload) — search / golden / bench-size
# parity, then an alternating A/B of the search line against the previous commit's library (prev).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r6l && export TMPDIR=/tmp
O=$R/gpurun_out/r6l
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_bench_sizes_gpu.py tests/test_golden.py tests/test_bench_launch_gpu.py tests/test_selfplay_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  for v in ${VARIANTS:-prev cur}; do
    unset MZ_LIB
    [ $v != cur ] && export MZ_LIB=$R/muzero.jl_amd/lib/libmz_$v.so
    timeout -k 10 300 python bench.py --no-cpu --search-only --steps 20 --warmup 3 > $O/ab_${v}_$i.log 2>&1 || { tail -20 $O/ab_${v}_$i.log; exit 1; }
    echo "$v $(tail -1 $O/ab_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('exp/s', round(d['value']/1e6,2), d['roofline']['kernel_ms'])")"
  done
done
