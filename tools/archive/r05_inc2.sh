#!/bin/bash
# Round 5: increments beside the chain (stream2) for CGMRES_P and the constrained suffix: tests,
# then C3 at tol 1e-7 and cgmres_p, increments on and off.
set -e
O=${1:-gpurun_out/r05inc2}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -k "incremental or k2s or golden or constraint_terms or restarted_cgmres or swe_vs_oracle_medium or cgmres_p or lkdvrk_gl3" -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || true
for inc in 1 0; do
  SPIS_GRAM_INC=$inc timeout -k 10 240 python -u bench.py --tol 1e-7 --steps 20 --no-cpu-baseline --no-cold > $O/c3_tol7_inc$inc.json 2> $O/c3_tol7_inc$inc.err
  SPIS_GRAM_INC=$inc timeout -k 10 240 python -u bench.py --method cgmres_p --steps 10 --no-cpu-baseline --no-cold > $O/c3_p_inc$inc.json 2> $O/c3_p_inc$inc.err
done
echo inc2-done
