#!/bin/bash
# K2s (one-pass small-N K2w): its tests, the golden suite, then C2 and the small-N sweep
set -e
O=${1:-gpurun_out/r04k2s}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "k2s or k2w_fold or golden or fused_dual" > $O/tests.log 2>&1
for M in 16667 33334 41667; do
  for v in "1 225000" "0 225000" "1 300000" "0 0"; do
    set -- $v
    SPIS_K2W_ONEPASS=$1 SPIS_K2W_SMALL_N=$2 timeout -k 10 200 python -u bench.py --config c2 --M $M --no-cpu-baseline --no-cold --steps 40 > $O/m${M}_$1_$2.json 2>> $O/err.log
    echo "M=$M onepass=$1 small_n=$2 $(python -c "import json; d=json.loads(open('$O/m${M}_$1_$2.json').read().strip().splitlines()[-1]); k=d['kernels']; print(round(d['value']), round(k.get('mgs_chain_us_mean',0),1), round(k.get('iteration_us',0),1), round(k.get('spmv_dual_us',0),1))")"
  done
done
echo k2s-done
