#!/bin/bash
# Round 5: the dual SpMV with one 16-B (x_j, z) pair gather per nonzero vs two 8-B gathers (kbench slab).
set -e
O=${1:-gpurun_out/r05pairs}
mkdir -p "$O"
timeout -k 10 300 python tools/dump_matrix.py 289 /tmp/kbench_mat > $O/dump3.txt 2>&1
timeout -k 10 200 ./tools/kbench /tmp/kbench_mat slab > $O/slab_c3.txt 2>&1
timeout -k 10 600 python tools/dump_matrix.py 913 /tmp/kbench_mat5 > $O/dump5.txt 2>&1
timeout -k 10 300 ./tools/kbench /tmp/kbench_mat5 slab > $O/slab_c5.txt 2>&1
echo pairs-done
