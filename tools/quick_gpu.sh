#!/bin/bash
# GPU iteration loop used during kernel work: small-kernel parity subset,
# phase stamps, bench.  Each GPU step has its own time limit; stops at the
# first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q \
    -k "${PARITY_K:-small or dispatch or golden or games}" > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 120 python tools/stamps.py --no-build > gpurun_out/st.log 2>&1 || { tail -20 gpurun_out/st.log; exit 1; }
tail -9 gpurun_out/st.log
timeout -k 10 200 python bench.py ${BENCH_ARGS} > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
tail -1 gpurun_out/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms', d['ms_per_step'], 'kernel', d['roofline']['kernel'], d['roofline']['kernel_ms'], 'learner', d['learner_steps_per_s'])"
