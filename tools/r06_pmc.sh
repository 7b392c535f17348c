#!/bin/bash
# Round 6: SpMV, MGS, transpose and K7t HBM traffic with provenance (GPU box): separate rocprofv3 --pmc passes, FETCH_SIZE then
# WRITE_SIZE, over tools/pmc_traffic.py run CFG (one counter group per pass, each under its own
# kill limit, MI355X_MICROARCH.md), then the reduction into gpurun_out/pmc_CFG/r06_traffic_CFG.json (copied to profiles/).
set -e
cfg=${1:-c3}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmc_$cfg
mkdir -p $out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $out/$c -o run -- \
    python tools/pmc_traffic.py run $cfg > $out/$c.log 2>&1
done
ff=$(find $out/FETCH_SIZE -name '*counter_collection.csv' | head -n 1)
fw=$(find $out/WRITE_SIZE -name '*counter_collection.csv' | head -n 1)
cp "$ff" $out/fetch.csv
cp "$fw" $out/write.csv
python tools/pmc_traffic.py reduce $cfg $out/fetch.csv $out/write.csv $out/r06_traffic_$cfg.json
echo done
