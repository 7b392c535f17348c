#!/bin/bash
# A/B of the slab key (SPIS_OPT_SLAB_KEY) on the GPU box: standalone SpMV sweep at C5 and C3, the
# C5 / C3 bench lines with the key off and on, then FETCH_SIZE / WRITE_SIZE passes of the C5 SpMVs
# with the key on (one counter group per pass, each under its own kill limit)
set -e
O=${1:-gpurun_out/slabkey}
mkdir -p "$O"
SPMV_SWEEP_KEYS=0,1 SPMV_SWEEP_NT=0 timeout -k 10 300 python -u tools/spmv_sweep.py 913 xcd > "$O/sweep913.log" 2>&1
SPMV_SWEEP_KEYS=0,1 SPMV_SWEEP_NT=0 timeout -k 10 120 python -u tools/spmv_sweep.py 289 xcd > "$O/sweep289.log" 2>&1
for k in 0 1; do
  timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline --slab-key $k > "$O/c5_k$k.log" 2>&1
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --slab-key $k > "$O/c3_k$k.log" 2>&1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d "$O/${c}_k1" -o run -- \
    python tools/spmv_pmc.py 913 0 1 1 > "$O/${c}_k1.log" 2>&1
done
echo done
