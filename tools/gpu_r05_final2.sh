#!/bin/bash
# Round 5, second final pass (after the one-player backup-chain change): the whole -m gpu suite,
# smoke(), the default bench line, the default command under --kernel-trace --stats, and configs[4].
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r5f3 && export TMPDIR=/tmp
O=$R/gpurun_out/r5f3
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
  > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/r05_final2_default_bench.json
python -c "import json; d=json.load(open('$O/r05_final2_default_bench.json')); print(d['value'], d['roofline']['frac'], d['learner_steps_per_s'], d['learner_steps_per_s_1step'], d['learner_roofline']['traffic'], d['train_loop']['node_expansions_per_s'], d['cpu_baseline']['value'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python bench.py --no-cpu > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
cp $O/kt/run_kernel_stats.csv $O/r05_final2_default_kernel_stats.csv
head -8 $O/r05_final2_default_kernel_stats.csv | cut -d, -f1-4
timeout -k 10 400 python bench.py --game atari > $O/atari.log 2>&1 || { echo "ATARI BENCH FAILED"; tail -20 $O/atari.log; exit 1; }
grep '^{' $O/atari.log | tail -1 > $O/r05_final2_atari_bench.json
python -c "import json; d=json.load(open('$O/r05_final2_atari_bench.json')); print('atari', d['value'], d['roofline']['frac'], d.get('learner_steps_per_s'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kta -o run -- python bench.py --game atari --no-cpu --search-only --steps 3 --warmup 1 > $O/profa.log 2>&1 || { tail -20 $O/profa.log; exit 1; }
cp $O/kta/run_kernel_stats.csv $O/r05_final2_atari_search_kernel_stats.csv
head -6 $O/r05_final2_atari_search_kernel_stats.csv | cut -d, -f1-4
