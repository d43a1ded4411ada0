#!/bin/bash
# Round 6 check of the tree: the whole GPU suite, smoke(), and the default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r6x && export TMPDIR=/tmp
O=$R/gpurun_out/r6x
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/bench.json
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'], d['learner_steps_per_s'], d['learner_steps_per_s_1step'], d['train_loop']['node_expansions_per_s'], (d.get('selfplay_pipeline') or {}).get('node_expansions_per_s'), d['cpu_baseline']['value'])"
