#!/bin/bash
# Round 5: K1w (windowed dual SpMV) vs K1dp in kbench, C3 and C5 matrices; window of 32 chunks
# (2 waves/SIMD), 16 chunks (2 and 3 waves/SIMD).
set -e
O=${1:-gpurun_out/r05win}
mkdir -p "$O"
timeout -k 10 300 python tools/dump_matrix.py 289 /tmp/kbench_mat > $O/dump3.txt 2>&1
for b in kbench kbench_w16 kbench_w16o3; do
  timeout -k 10 200 ./tools/$b /tmp/kbench_mat win > $O/win_c3_$b.txt 2>&1
done
timeout -k 10 600 python tools/dump_matrix.py 913 /tmp/kbench_mat5 > $O/dump5.txt 2>&1
for b in kbench kbench_w16 kbench_w16o3; do
  timeout -k 10 300 ./tools/$b /tmp/kbench_mat5 win > $O/win_c5_$b.txt 2>&1
done
echo win-done
