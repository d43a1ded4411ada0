#!/bin/bash
# Rehearse the N > 1 bench path on a one-GPU box: 2 ranks on cuda:0 over gloo
# (RCCL needs one GPU per rank; the driver's 8-GPU run uses it).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)} && mkdir -p gpurun_out
for a in "" "--net resnet --games 256" "--game connect4 --games 128"; do
  MZ_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu $a \
    > gpurun_out/dp.log 2>&1 || { tail -30 gpurun_out/dp.log; exit 1; }
  grep '^{' gpurun_out/dp.log | tail -1 | cut -c1-400
done
