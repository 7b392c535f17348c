#!/bin/bash
# Round-3 profiles (GPU box): kernel-trace summaries of the 1-rank distributed C3 bench and of the
# C5 bench, then FETCH_SIZE / WRITE_SIZE PMC passes of the C5 bench (one counter group per pass).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof3
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3/dist1 -o run -- \
  python bench.py --force-distributed --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof3/dist1.log 2>&1
unset MASTER_ADDR MASTER_PORT RANK LOCAL_RANK WORLD_SIZE
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3/c5 -o run -- \
  python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-cold > gpurun_out/prof3/c5.log 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/prof3/pmc_$c -o run -- \
    python bench.py --config c5 --steps 1 --warmup 0 --cycles 2 --no-cpu-baseline --no-cold > gpurun_out/prof3/pmc_$c.log 2>&1
done
echo done
