#!/bin/bash
# SPIS_OPT_C16_TM: its parity tests, the standalone SpMV sweep (16-bit columns) at C5 / C3 with the
# copy off and on, then the C5 bench both ways
set -e
O=${1:-gpurun_out/tm}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "thread_major or col16_bit or w4" > "$O/tests.log" 2>&1
SPMV_SWEEP_TM=0,1 SPMV_SWEEP_NT=0 timeout -k 10 300 python -u tools/spmv_sweep.py 913 xcd > "$O/sweep913.log" 2>&1
SPMV_SWEEP_TM=0,1 SPMV_SWEEP_NT=0 timeout -k 10 120 python -u tools/spmv_sweep.py 289 xcd > "$O/sweep289.log" 2>&1
for t in 0 1; do
  timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline --c16-tm $t > "$O/c5_tm$t.log" 2>&1
done
echo done
