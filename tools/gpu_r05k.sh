#!/bin/bash
# Round 5: inputs of the configs[1] latency model — the stage probe (five modes) and the
# per-phase stamps of mz_search_small2 at the bench launch (G = 512, S = 50).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r5k && export TMPDIR=/tmp
O=$R/gpurun_out/r5k
timeout -k 10 60 ./tools/barrier_probe > $O/barrier_probe.txt 2>&1 || { cat $O/barrier_probe.txt; exit 1; }
cat $O/barrier_probe.txt
timeout -k 10 200 python tools/stamps.py --no-build > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
grep -v amdgpu $O/stamps.txt | tail -25
