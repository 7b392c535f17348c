#!/bin/bash
# Round 5, K2q counted waits: chainbench A/B (CW vs the vmcnt(0) build of the same kernel), the
# CW chain's phase trace, the chain / golden parity tests, then the C3 and C4 bench lines.
set -e
O=${1:-gpurun_out/r05cw}
mkdir -p "$O"
timeout -k 10 120 ./tools/chainbench 1002252 20 ring > $O/ring.txt 2>&1
timeout -k 10 120 ./tools/chainbench 1002252 20 trace > $O/trace.txt 2>&1
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -k "chain or golden or full_size_swe_c3 or fused_dual" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 240 python -u bench.py --no-cpu-baseline > $O/c3a.json 2> $O/c3a.err
timeout -k 10 240 python -u bench.py --no-cpu-baseline > $O/c3b.json 2> $O/c3b.err
timeout -k 10 240 python -u bench.py --config c4 --no-cpu-baseline > $O/c4.json 2> $O/c4.err
echo cw-done
