#!/bin/bash
# HBM traffic of the fused dual SpMV (K1dp) from two separate rocprofv3 --pmc passes of
# tools/kbench's pmc mode (MI355X_MICROARCH.md: one counter group per pass), then the summary
# json via tools/pmc_dual.py.  usage (GPU box): tools/pmc_dual.sh TAG
set -e
tag=${1:-r02}
python tools/dump_matrix.py 289 /tmp/kbench_mat
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_$c -o run -- tools/kbench /tmp/kbench_mat pmc
  f=$(find gpurun_out/pmc_$c -name '*counter_collection.csv' | head -n 1)
  cp "$f" gpurun_out/${tag}_pmc_$(echo $c | tr A-Z a-z).csv
done
