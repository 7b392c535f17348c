#!/bin/bash
# A/B of the round-4 cache knobs (measurement only): K2q's temporal basis window (SPIS_EXP_TW) at
# C3, K2w's temporal dot pass + reversed update (SPIS_EXP_REV) at C5 and through the several-GPU
# path at one rank.  Each run has its own time limit; set -e stops at the first failure.
set -e
O=${1:-gpurun_out/r04ab}
mkdir -p "$O"
for tw in 0 6 10 0 6; do
  SPIS_EXP_TW=$tw timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-cold --steps 30 > $O/c3_tw$tw.json 2>> $O/err.log
  tail -1 $O/c3_tw$tw.json | cut -c1-120
done
for rv in 0 1; do
  SPIS_EXP_REV=$rv timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --no-cold --steps 3 --warmup 1 > $O/c5_rev$rv.json 2>> $O/err.log
  SPIS_EXP_REV=$rv timeout -k 10 200 python -u bench.py --force-distributed --no-cpu-baseline --no-cold --steps 30 > $O/dist1_rev$rv.json 2>> $O/err.log
done
echo ab-done
