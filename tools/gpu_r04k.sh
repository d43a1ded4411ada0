#!/bin/bash
# Corrected-learner tests, the FC / Connect4 corrected-learner stamps, then the
# Atari line (corrected leg through the downsampler) under kernel-trace stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r4k && export TMPDIR=/tmp
O=$R/gpurun_out/r4k
timeout -k 10 300 python -u -m pytest tests/test_corrected_resnet_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 200 python tools/bp_stamps.py > $O/bp_stamps.log 2>&1 || { tail -20 $O/bp_stamps.log; exit 1; }
cat $O/bp_stamps.log
NET=resnet GAME=connect4 timeout -k 10 200 python tools/bp_stamps.py > $O/rbp_stamps.log 2>&1 || { tail -20 $O/rbp_stamps.log; exit 1; }
head -c 3000 $O/rbp_stamps.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_atari -o run -- python bench.py --game atari --no-cpu > $O/atari.log 2>&1 || { tail -20 $O/atari.log; exit 1; }
grep '^{' $O/atari.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['learner_steps_per_s'], d['learner_corrected'])"
head -14 $O/kt_atari/run_kernel_stats.csv | cut -d, -f1-4
