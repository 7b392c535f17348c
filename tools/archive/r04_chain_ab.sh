#!/bin/bash
# K2q change check: the chain tests, then the C3 bench twice (chain mean and it/s).
set -e
O=${1:-gpurun_out/r04ab}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "chain or golden or full_size_swe_c3 or fused_dual" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 240 python -u bench.py --no-cpu-baseline > $O/c3a.json 2> $O/c3a.err
timeout -k 10 240 python -u bench.py --no-cpu-baseline > $O/c3b.json 2> $O/c3b.err
timeout -k 10 240 python -u bench.py --config c4 --no-cpu-baseline > $O/c4.json 2> $O/c4.err
echo ab-done
