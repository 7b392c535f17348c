#!/bin/bash
# the several-GPU code path at one rank (self-halo tests, --force-distributed bench) after the merged
# residual + dot all-reduce; then C3 on 32- vs 16-bit columns, alternating
set -e
O=${1:-gpurun_out/call4}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "self_halo or distributed" > "$O/dist_tests.log" 2>&1
timeout -k 10 240 python -u bench.py --force-distributed --no-cpu-baseline > "$O/dist1.log" 2>&1
for r in 1 2; do
  for c in 1 2; do
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-cold --col16 $c > "$O/c3_col$c_$r.log" 2>&1
    cp "$O/c3_col$c_$r.log" "$O/c3_col${c}_r$r.log"
  done
done
echo done
