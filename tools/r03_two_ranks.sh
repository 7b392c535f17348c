#!/bin/bash
# Rehearsal of the several-GPU path on a one-GPU box: two ranks pinned to device 0 (SPIS_DEVICE),
# RCCL between them, C3 weak-scaling and C4 strong-scaling bench lines, each under its own limit
set -e
O=${1:-gpurun_out/r2}
mkdir -p "$O"
export SPIS_DEVICE=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline > "$O/c3.log" 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29512 bench.py --gpus 2 --config c4 --steps 5 --warmup 1 --no-cpu-baseline > "$O/c4.log" 2>&1
echo done
