#!/bin/bash
# Round 6 final tree: per-phase stamps of mz_search_small2 at the configs[1] launch, with the per-wave split of
# the post-network phase (wave 0 read-outs + backup, wave 2 expand, wave 3 h' store).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r6af && export TMPDIR=/tmp
O=$R/gpurun_out/r6af
timeout -k 10 200 python tools/stamps.py --no-build > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
grep -v amdgpu.ids $O/stamps.txt
