#!/bin/bash
# Round 5: r0 without the matrix when x0 = 0: tests, C3 and C5 benches, C3 timeline.
O=${1:-gpurun_out/r05x0}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -k "x0_zero or golden or restarted or swe_vs_oracle_medium or full_size_swe_c3 or edge" -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stop"; exit $rc; fi
set -e
timeout -k 10 240 python -u bench.py --no-cold --no-cpu-baseline > $O/c3.json 2> $O/c3.err
timeout -k 10 240 python -u bench.py --no-cold --no-cpu-baseline > $O/c3b.json 2> $O/c3b.err
timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cold --no-cpu-baseline > $O/c5.json 2> $O/c5.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 6 --warmup 1 --no-cpu-baseline --no-cold > $O/prof.json 2> $O/prof.err
f=$(find $O/prof -name '*kernel_trace.csv' | head -n 1)
(cd tools && python trace_timeline.py ../$f 600) > $O/timeline.txt
echo x0-done
