#!/bin/bash
# Several ranks on one GPU through the host transport (SPIS_TRANSPORT=host): the multi-rank GPU
# tests, the 1-rank RCCL self-halo tests, and bench.py --gpus 2 / 4 under torch.distributed.run
# (every rank on GPU 0; the numbers exercise the code path, they are not a scaling measurement).
set -e
O=${1:-gpurun_out/r04mr}
mkdir -p "$O"
timeout -k 10 700 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_parity.py -k "several_ranks or self_halo" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
for P in 2 4; do
  SPIS_DEVICE=0 SPIS_TRANSPORT=host timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $P --master-addr 127.0.0.1 --master-port $((29500 + P)) bench.py --gpus $P --steps 3 --warmup 1 --no-cpu-baseline > $O/bench$P.json 2> $O/bench$P.err
done
echo multirank-done
