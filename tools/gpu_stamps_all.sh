#!/bin/bash
# Phase / per-layer stamps from the prebuilt -DMZ_STAMPS library (libmz_stamps.so):
# FC search (small2), ResNet search networks, ResNet learner chain.  Each step has its
# own limit; the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 120 python tools/stamps.py --no-build > gpurun_out/st_fc.log 2>&1 || { tail -20 gpurun_out/st_fc.log; exit 1; }
tail -12 gpurun_out/st_fc.log
timeout -k 10 120 python tools/rn_chain_stamps.py --no-build > gpurun_out/st_chain.log 2>&1 || { tail -20 gpurun_out/st_chain.log; exit 1; }
cat gpurun_out/st_chain.log
timeout -k 10 120 python tools/rn_stamps.py --no-build > gpurun_out/st_rn.log 2>&1 || { tail -20 gpurun_out/st_rn.log; exit 1; }
cat gpurun_out/st_rn.log
