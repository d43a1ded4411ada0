#!/bin/bash
# Round 6 (f32 tanh adopted): the whole -m gpu suite and smoke(), then the default line's profiles
# (tools/gpu_r02_profiles.sh with TAG=r06m: kernel-trace stats, FETCH / WRITE / SQ passes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r6m && export TMPDIR=/tmp
O=$R/gpurun_out/r6m
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
TAG=r06m SKIP_RESNET=1 SKIP_ATARI=1 bash tools/gpu_r02_profiles.sh > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
python -c "
import json
d=json.load(open('gpurun_out/rp/r06m_default_bench_under_rocprof.json'))
print(d['value'], d['roofline']['frac'], d['learner_steps_per_s'], d['learner_steps_per_s_1step'], d['train_loop']['node_expansions_per_s'])
p=json.load(open('gpurun_out/rp/pmc2_r06m_default.json'))['kernels']
for k,v in p.items(): print(k, v.get('hbm_bytes_per_launch_fetch_x2'), v.get('wait_any_frac'), v.get('dispatches'))
"
head -8 gpurun_out/rp/r06m_default_kernel_stats.csv | cut -d, -f1-4
