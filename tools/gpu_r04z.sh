#!/bin/bash
# Round-4 final tree: the whole -m gpu suite, smoke, the default bench line (CPU
# baseline included) under kernel-trace stats, and the ResNet / Connect4 / Atari
# lines.  Each GPU step has its own limit; the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r4z && export TMPDIR=/tmp
O=$R/gpurun_out/r4z
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_default -o run -- python bench.py > $O/default.log 2>&1 || { tail -20 $O/default.log; exit 1; }
grep '^{' $O/default.log | tail -1 > $O/r04z_default_bench_under_rocprof.json
head -8 $O/kt_default/run_kernel_stats.csv | cut -d, -f1-4
timeout -k 10 300 python bench.py > $O/default_clean.log 2>&1 || { tail -20 $O/default_clean.log; exit 1; }
grep '^{' $O/default_clean.log | tail -1 > $O/r04z_config1_bench.json
python -c "import json; d=json.load(open('$O/r04z_config1_bench.json')); print('config1', d['value'], d['roofline']['frac'], d['learner_steps_per_s'], d['learner_corrected']['learner_steps_per_s'], d['cpu_baseline']['value'])"
for c in resnet connect4 atari; do
  case $c in resnet) A="--net resnet";; connect4) A="--game connect4 --net resnet";; atari) A="--game atari";; esac
  timeout -k 10 400 python bench.py $A --no-cpu > $O/$c.log 2>&1 || { tail -20 $O/$c.log; exit 1; }
  grep '^{' $O/$c.log | tail -1 > $O/r04z_${c}_bench.json
  python -c "import json; d=json.load(open('$O/r04z_${c}_bench.json')); print('$c', d['value'], d['roofline']['frac'], d['learner_steps_per_s'], d['learner_corrected']['learner_steps_per_s'])"
done
