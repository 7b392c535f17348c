#!/bin/bash
# K2w (two-pass one-reduce MGS) against K2q on one GPU at small N: lkdv (C2's operator) at
# N = 100 k .. 300 k, K2q forced by SPIS_K2W_SMALL_N=0
set -e
O=${1:-gpurun_out/r04k2ws2}
mkdir -p "$O"
for M in 16667 25000 33334 41667 50000; do
  for sm in 0 1000000 0 1000000; do
    SPIS_K2W_SMALL_N=$sm timeout -k 10 200 python -u bench.py --config c2 --M $M --no-cpu-baseline --no-cold --steps 40 > $O/m${M}_$sm.json 2>> $O/err.log
    echo "M=$M small_n=$sm $(python -c "import json; d=json.loads(open('$O/m${M}_$sm.json').read().strip().splitlines()[-1]); k=d['kernels']; print(round(d['value']), round(k.get('mgs_chain_us_mean',0),1), round(k.get('iteration_us',0),1))")"
  done
done
echo k2ws-done
