#!/bin/bash
# Round 5: incremental constraint Gram + contraction-off one-reduce kernels: their tests and the
# golden suite, the K2s/K2w bitwise diff at 196,608, then C3 at tol 1e-7 and cgmres_p with the
# increments on and off, and the default C3 line.
set -e
O=${1:-gpurun_out/r05inc}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -k "incremental or k2s or golden or constraint_terms or restarted_cgmres or swe_vs_oracle_medium or cgmres_p" -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || true
timeout -k 10 200 python -u tools/r04_k2s_diff.py > $O/k2s_diff.txt 2>&1 || true
for inc in 1 0; do
  SPIS_GRAM_INC=$inc timeout -k 10 240 python -u bench.py --tol 1e-7 --steps 20 --no-cpu-baseline --no-cold > $O/c3_tol7_inc$inc.json 2> $O/c3_tol7_inc$inc.err
  SPIS_GRAM_INC=$inc timeout -k 10 240 python -u bench.py --method cgmres_p --steps 10 --no-cpu-baseline --no-cold > $O/c3_p_inc$inc.json 2> $O/c3_p_inc$inc.err
done
timeout -k 10 240 python -u bench.py --no-cpu-baseline > $O/c3.json 2> $O/c3.err
echo inc-done
