#!/bin/bash
# C2 / C4 SpMV HBM traffic (GPU box): separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over
# tools/spmv_pmc.py (standalone, back to back as in the solver), one counter group per pass
# (MI355X_MICROARCH.md), each under its own kill limit; then per-kernel MB by tools/pmc_kernels.py
# with the r02c calibration streams
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc4
for cfg in c2 c4; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc4/${cfg}_$c -o run -- \
      python tools/spmv_pmc.py $cfg 0 0 > gpurun_out/pmc4/${cfg}_$c.log 2>&1
    f=$(find gpurun_out/pmc4/${cfg}_$c -name '*counter_collection.csv' | head -n 1)
    cp "$f" gpurun_out/pmc4/r03_${cfg}_pmc_$(echo $c | tr A-Z a-z).csv
  done
  python tools/pmc_kernels.py gpurun_out/pmc4/r03_${cfg}_pmc_fetch_size.csv gpurun_out/pmc4/r03_${cfg}_pmc_write_size.csv \
    profiles/r02c_pmc_fetch_size.csv profiles/r02c_pmc_write_size.csv gpurun_out/pmc4/r03_${cfg}_spmv_traffic.json
done
echo done
