#!/bin/bash
# Round-3 measurement pass: default bench line, the search-only command under rocprofv3 (its
# mz_search_small2 average is the bench's timed searches alone), the self-launched 2-rank gloo
# rehearsal (bench.py --gpus 2 with no torchrun), each GPU step under its own time limit.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)} && mkdir -p gpurun_out/m3 && export TMPDIR=/tmp
O=gpurun_out/m3
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_search -o run -- python bench.py --search-only --no-cpu > $O/bench_search.log 2>&1 || { tail -20 $O/bench_search.log; exit 1; }
tail -1 $O/bench_search.log
find $O/kt_search -name '*kernel_stats.csv' -exec head -5 {} \;
MZ_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --no-cpu --train-moves 0 > $O/bench_gloo2.log 2>&1 || { tail -30 $O/bench_gloo2.log; exit 1; }
grep '^{' $O/bench_gloo2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('n_gpus', d['n_gpus'], 'value', d['value'], 'learner', d['learner_steps_per_s'], d['learner_config']['batch_source'])"
