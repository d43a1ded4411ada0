#!/bin/bash
# Round 6: per-phase stamps (-DMZ_STAMPS library built on the CPU side) of mz_search_small2 at the
# configs[1] launch, with the tail schedule and without it (MZ_NO_TAIL=1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r6b && export TMPDIR=/tmp
O=$R/gpurun_out/r6b
timeout -k 10 200 python tools/stamps.py --no-build > $O/stamps_tail.txt 2>&1 || { tail -20 $O/stamps_tail.txt; exit 1; }
cat $O/stamps_tail.txt
MZ_NO_TAIL=1 timeout -k 10 200 python tools/stamps.py --no-build > $O/stamps_notail.txt 2>&1 || { tail -20 $O/stamps_notail.txt; exit 1; }
cat $O/stamps_notail.txt
