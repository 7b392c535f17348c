#!/bin/bash
# Round 5: K2s with two chunks per workgroup (N up to 524,288): parity test, C4 with it (default)
# and with K2q (SPIS_K2W_SMALL_N=0), C2 unchanged.
O=${1:-gpurun_out/r05k2s2}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "k2s" -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stop"; exit $rc; fi
set -e
timeout -k 10 240 python -u bench.py --config c4 --steps 30 --no-cpu-baseline --no-cold > $O/c4.json 2> $O/c4.err
SPIS_K2W_SMALL_N=0 timeout -k 10 240 python -u bench.py --config c4 --steps 30 --no-cpu-baseline --no-cold > $O/c4_k2q.json 2> $O/c4_k2q.err
timeout -k 10 240 python -u bench.py --config c4 --steps 30 --no-cpu-baseline --no-cold > $O/c4_again.json 2> $O/c4_again.err
timeout -k 10 240 python -u bench.py --config c2 --steps 30 --no-cpu-baseline --no-cold > $O/c2.json 2> $O/c2.err
echo k2s2-done
