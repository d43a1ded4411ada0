#!/bin/bash
# Round-4 first box: the whole -m gpu suite, smoke, the default and ResNet bench
# lines, then FETCH_SIZE / WRITE_SIZE passes of the ResNet line for the network
# launch's traffic (each counter in its own rocprofv3 run).  Each GPU step has
# its own limit; the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r4 && export TMPDIR=/tmp
O=$R/gpurun_out/r4
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 ${TEST_TIMEOUT:-800} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
fi
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('config1', d['value'], d['roofline']['frac'], 'learner', d['learner_steps_per_s'], d['cpu_baseline'])"
timeout -k 10 400 python bench.py --net resnet --no-cpu > $O/bench_resnet.log 2>&1 || { tail -20 $O/bench_resnet.log; exit 1; }
grep '^{' $O/bench_resnet.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('config2', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], 'learner', d['learner_steps_per_s'])"
B="--net resnet --steps 4 --warmup 1 --no-cpu --pipeline-moves 0 --train-moves 0 --learner-steps 10"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $O/rn_$c -o run -- python bench.py $B > $O/rn_$c.log 2>&1 || { echo FAILED $c; tail -5 $O/rn_$c.log; exit 1; }
done
python tools/pmc_kernels.py $O/pmc2_r04a_resnet.json "python bench.py $B" $O/rn_FETCH_SIZE $O/rn_WRITE_SIZE -- \
    mz_rsearch_nets mz_runroll_fused_r mz_rsearch_tree_lds mz_rsearch_root > /dev/null
python -c "import json; d=json.load(open('$O/pmc2_r04a_resnet.json')); print({k: (round(v['FETCH_SIZE']), round(v['WRITE_SIZE']), v.get('hbm_bytes_per_launch_fetch_x2')) for k, v in d['kernels'].items()})"
