#!/bin/bash
# 2,048- vs 4,096-nnz row blocks for the dual SpMV (tools/kbench cap4k) at C5 and C3, then the
# counter list and an SQ wave-state pass over the C5 SpMV launches
set -e
O=${1:-gpurun_out/cap4k}
mkdir -p "$O"
timeout -k 10 200 python tools/dump_matrix.py 913 /tmp/km913 > "$O/dump.log" 2>&1
timeout -k 10 200 ./tools/kbench /tmp/km913 cap4k > "$O/c5.log" 2>&1
timeout -k 10 100 python tools/dump_matrix.py 289 /tmp/km289 >> "$O/dump.log" 2>&1
timeout -k 10 100 ./tools/kbench /tmp/km289 cap4k > "$O/c3.log" 2>&1
bash tools/r03_pmc_sq.sh "$O/pmcsq"
