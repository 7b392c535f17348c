#!/bin/bash
# SPIS_OPT_SPMV_W4 = 2 (buffer-descriptor SpMV at 3 waves per SIMD): parity tests, the standalone
# sweep at C5 / C3 against the default, then C3 and C5 bench lines both ways
set -e
O=${1:-gpurun_out/buf}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "w4 or pipe_modes" > "$O/tests.log" 2>&1
SPMV_SWEEP_W4=0,2 SPMV_SWEEP_NT=0 timeout -k 10 300 python -u tools/spmv_sweep.py 913 xcd > "$O/sweep913.log" 2>&1
SPMV_SWEEP_W4=0,2 SPMV_SWEEP_NT=0 timeout -k 10 120 python -u tools/spmv_sweep.py 289 xcd > "$O/sweep289.log" 2>&1
for w in 0 2 0 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-cold --spmv-w4 $w > "$O/c3_w$w.log" 2>&1
  cat "$O/c3_w$w.log" >> "$O/c3_all_w$w.log"
done
for w in 0 2; do
  timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline --no-cold --spmv-w4 $w > "$O/c5_w$w.log" 2>&1
done
echo done
