#!/bin/bash
# A/B of library variants (MZ_LIB, $LIBS; "base" = the in-tree libmz.so) on the corrected
# ResNet learner: bench.py's learner_corrected leg for TicTacToe ResNet and Connect4 ResNet-8.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
for n in ${LIBS:-base}; do
  if [ "$n" = base ]; then unset MZ_LIB; else export MZ_LIB=$R/muzero.jl_amd/lib/libmz_$n.so; fi
  for g in tictactoe connect4; do
    timeout -k 10 200 python bench.py --game $g --net resnet --no-cpu --steps 2 --warmup 1 --pipeline-moves 0 --train-moves 0 --learner-steps 10 > gpurun_out/abr_$n.log 2>&1 || { tail -20 gpurun_out/abr_$n.log; exit 1; }
    echo "$n $g $(grep -o '"learner_corrected": {[^}]*}' gpurun_out/abr_$n.log | cut -c1-90)"
  done
done
