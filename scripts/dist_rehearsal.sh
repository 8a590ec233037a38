#!/bin/bash
# Rehearse the N>1 bench path on a one-GPU box: 2 ranks share cuda:0, gradients all-reduced over
# gloo (RCCL needs distinct GPUs).  Throughput is not meaningful; the run checks the path end to end.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
GSR_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 \
  --no-cpu-baseline > gpurun_out/dist2.json 2> gpurun_out/dist2.err
rc=$?; echo "dist rc=$rc"; cat gpurun_out/dist2.json; tail -5 gpurun_out/dist2.err; exit $rc
