#!/bin/bash
# configs[3] learner A/B: one-column-block units for the ResNet chain (MZ_RN_CHAIN_NB1=1),
# its parity test with the switch on, then alternating bench lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r4d && export TMPDIR=/tmp
O=$R/gpurun_out/r4d
MZ_RN_CHAIN_NB1=1 timeout -k 10 300 python -u -m pytest tests/test_bench_sizes_gpu.py tests/test_resnet_gpu.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
B="--game connect4 --net resnet --no-cpu --steps 3 --warmup 1 --pipeline-moves 0 --train-moves 0 --learner-steps 60"
for i in 1 2; do
  for v in base nb1; do
    if [ $v = nb1 ]; then export MZ_RN_CHAIN_NB1=1; else unset MZ_RN_CHAIN_NB1; fi
    timeout -k 10 300 python bench.py $B > $O/$v$i.log 2>&1 || { tail -20 $O/$v$i.log; exit 1; }
    grep '^{' $O/$v$i.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['learner_steps_per_s'], d.get('learner_roofline',{}).get('kernel'))"
  done
done
