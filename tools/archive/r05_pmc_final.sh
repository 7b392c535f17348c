#!/bin/bash
# Round 5, final: PMC traffic at HEAD for C3, C2, C4, C5, then the bench lines that quote it.
set -e
bash tools/r05_pmc_all.sh
for c in c3 c2 c4 c5; do cp gpurun_out/pmc_$c/r05_traffic_$c.json profiles/; done
mkdir -p gpurun_out/r05pf
timeout -k 10 240 python -u bench.py > gpurun_out/r05pf/c3.json 2> gpurun_out/r05pf/c3.err
timeout -k 10 240 python -u bench.py --config c2 > gpurun_out/r05pf/c2.json 2> gpurun_out/r05pf/c2.err
timeout -k 10 240 python -u bench.py --config c4 > gpurun_out/r05pf/c4.json 2> gpurun_out/r05pf/c4.err
timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 1 > gpurun_out/r05pf/c5.json 2> gpurun_out/r05pf/c5.err
cp profiles/r05_traffic_*.json gpurun_out/r05pf/
echo pmc-final-done
