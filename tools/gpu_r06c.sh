#!/bin/bash
# Round 6: tail layout one wave per SIMD — stamps (tail / no tail), then alternating A/B of the default
# bench line: HEAD~ round-5 library (libmz_head.so), this library with and without the tail.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r6c && export TMPDIR=/tmp
O=$R/gpurun_out/r6c
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_bench_sizes_gpu.py tests/test_golden.py -k "small or configs1 or golden or games" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python tools/stamps.py --no-build > $O/stamps_tail.txt 2>&1 || { tail -20 $O/stamps_tail.txt; exit 1; }
grep -E "nets|expand|backup|total" $O/stamps_tail.txt
for i in 1 2; do
  for v in head tail notail; do
    unset MZ_LIB MZ_NO_TAIL
    [ $v = head ] && export MZ_LIB=$R/muzero.jl_amd/lib/libmz_head.so
    [ $v = notail ] && export MZ_NO_TAIL=1
    timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 3 --pipeline-moves 10 --train-moves 0 > $O/ab_${v}_$i.log 2>&1 || { tail -20 $O/ab_${v}_$i.log; exit 1; }
    echo "$v $(tail -1 $O/ab_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('exp/s', round(d['value']/1e6,2), d['roofline']['kernel'], d['roofline']['kernel_ms'], 'learner', d['learner_steps_per_s'], 'pipe', round(d['selfplay_pipeline']['node_expansions_per_s']/1e6,2))")"
  done
done
