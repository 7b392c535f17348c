#!/bin/bash
# K2w fold / temporal window: GPU tests, then A/B through the several-GPU path at one rank and C5.
set -e
O=${1:-gpurun_out/r04fold}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "k2w_fold or self_halo or mgs_chain_matches" > $O/tests.log 2>&1
for v in "1 -1" "0 -1" "1 0" "0 0" "1 -1" "0 -1"; do
  set -- $v
  if [ "$2" = "-1" ]; then unset SPIS_K2W_TW; else export SPIS_K2W_TW=$2; fi
  SPIS_K2W_FOLD=$1 timeout -k 10 200 python -u bench.py --force-distributed --no-cpu-baseline --no-cold --steps 30 > $O/d1_f$1_tw$2.json 2>> $O/err.log
  echo "fold=$1 tw=$2 $(tail -1 $O/d1_f$1_tw$2.json | cut -c1-110)"
done
unset SPIS_K2W_TW
for f in 1 0; do
  SPIS_K2W_FOLD=$f timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --no-cold --steps 3 --warmup 1 > $O/c5_f$f.json 2>> $O/err.log
  echo "c5 fold=$f $(tail -1 $O/c5_f$f.json | cut -c1-110)"
done
echo fold-done
