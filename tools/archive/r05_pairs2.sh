#!/bin/bash
# Round 5: the chain writes (x_j, q_{j+2}) pairs, the dual SpMV gathers them: tests, C3 benches,
# chainbench ring (the chain kernel's cost of the extra stores).
O=${1:-gpurun_out/r05pairs2}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -k "golden or fused or dual or spmv or swe_vs_oracle_medium or full_size_swe_c3 or incremental" -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stop"; exit $rc; fi
set -e
timeout -k 10 240 python -u bench.py --no-cold --no-cpu-baseline > $O/c3.json 2> $O/c3.err
timeout -k 10 240 python -u bench.py --no-cold --no-cpu-baseline > $O/c3b.json 2> $O/c3b.err
timeout -k 10 240 python -u bench.py --config c4 --no-cold --no-cpu-baseline > $O/c4.json 2> $O/c4.err
timeout -k 10 200 ./tools/chainbench 1002252 20 ring > $O/ring.txt 2>&1
CHAINBENCH_XZ=0 timeout -k 10 200 ./tools/chainbench 1002252 20 ring > $O/ring_noxz.txt 2>&1
echo pairs2-done
