#!/bin/bash
# C5 SpMV HBM traffic (GPU box): separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over
# tools/spmv_pmc.py, one counter group per pass (MI355X_MICROARCH.md), each under its own kill limit
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc3
nt=${1:-0}
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc3/${c}_nt$nt -o run -- \
    python tools/spmv_pmc.py 913 $nt > gpurun_out/pmc3/${c}_nt$nt.log 2>&1
  f=$(find gpurun_out/pmc3/${c}_nt$nt -name '*counter_collection.csv' | head -n 1)
  cp "$f" gpurun_out/pmc3/r03_c5_pmc_$(echo $c | tr A-Z a-z)_nt$nt.csv
done
echo done
