#!/bin/bash
# Round 5: the downsampler with compile-time 3x3 taps (Atari / configs[4]) and
# the FC corrected learner's specialised dW jobs — parity tests, then the
# configs[4] bench line + kernel stats, then the FC corrected leg.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r5e && export TMPDIR=/tmp
O=$R/gpurun_out/r5e
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_atari_gpu.py tests/test_corrected_resnet_gpu.py tests/test_corrected_learner_gpu.py tests/test_fc_bn.py \
  "tests/test_bench_launch_gpu.py::test_configs4_atari_512x200" > $O/tests.log 2>&1 \
  || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --game atari --no-cpu > $O/atari.log 2>&1 || { echo "FAILED atari"; tail -5 $O/atari.log; exit 1; }
grep '^{' $O/atari.log | tail -1 > $O/r05e_atari_bench.json
python -c "import json; d=json.load(open('$O/r05e_atari_bench.json')); print('atari', d['value'], d['learner_steps_per_s'], (d['learner_corrected'] or {}).get('learner_steps_per_s'), d['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_atari -o run -- python bench.py --game atari --no-cpu --pipeline-moves 0 --train-moves 0 > $O/prof_atari.log 2>&1 || { tail -5 $O/prof_atari.log; exit 1; }
head -12 $O/kt_atari/run_kernel_stats.csv | cut -d, -f1-4
grep -h "downsample\|dsbp" $O/kt_atari/run_kernel_stats.csv | cut -d, -f1-4
timeout -k 10 200 python bench.py --no-cpu --pipeline-moves 0 --steps 5 --train-moves 0 --learner-chunk 1 > $O/fc.log 2>&1 || { echo "FAILED fc"; tail -5 $O/fc.log; exit 1; }
grep '^{' $O/fc.log | tail -1 > $O/fc.json
python -c "import json; d=json.load(open('$O/fc.json')); c=d['learner_corrected']; print('fc corrected', c['learner_steps_per_s'], c['step_ms'])"
MZ_LIB=$R/muzero.jl_amd/lib/libmz_stamps.so timeout -k 10 120 python tools/ds_stamps.py 32 2>&1 | grep -v amdgpu.ids | tail -22
