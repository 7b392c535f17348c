#!/bin/bash
# Round 5: the several-rank bench path after the warm-up change: 2 ranks on one GPU over the host
# transport (rehearsal; RCCL refuses two ranks on one device), and the one-rank RCCL path.
set -e
O=${1:-gpurun_out/r05d2}
mkdir -p "$O"
SPIS_DEVICE=0 SPIS_TRANSPORT=host timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > $O/g2.json 2> $O/g2.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 1 --force-distributed --steps 10 --warmup 2 > $O/g1.json 2> $O/g1.err
echo d2-done
