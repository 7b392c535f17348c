#!/bin/bash
# Round 5: the multi-rank GPU tests (C3/C2 shapes at 2 and 4 ranks, C4's split at 4, C5's at 8
# ranks restarted), the C5 cycle-0 full-size test with its arm logged, then the C3 bench line.
set -e
O=${1:-gpurun_out/r05mr}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py -v -s --timeout 400 --timeout-method thread -p no:cacheprovider > $O/multirank.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/c3.json 2> $O/c3.err
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "c5_cycle0" -x -v -s --timeout 500 --timeout-method thread -p no:cacheprovider > $O/c5c0.log 2>&1
echo r05mr-done
