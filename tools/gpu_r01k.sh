#!/bin/bash
# Final round-1 measurements: round profiles (tools/gpu_round_profiles.sh) plus the configs[0]
# single-game lines (G=1, S=25 and the shipped S=10) that SURVEY §8d config 1 asks for.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)} && mkdir -p gpurun_out/rp
T=${TAG:-r01k}
TAG=$T bash tools/gpu_round_profiles.sh || exit 1
for s in 25 10; do
  timeout -k 10 300 python bench.py --games 1 --sims $s --pipeline-moves 0 > gpurun_out/rp/${T}_config1_s$s.log 2>&1 \
    || { tail -20 gpurun_out/rp/${T}_config1_s$s.log; exit 1; }
  grep '^{' gpurun_out/rp/${T}_config1_s$s.log | tail -1 > gpurun_out/rp/${T}_config1_s${s}_bench.json
done
