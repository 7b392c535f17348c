#!/bin/bash
# Round 5: C3 with U_{k-2}'s residual during the host KKT, kernel trace timeline, host overhead profile.
set -e
O=${1:-gpurun_out/r05host}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "golden or paired or residual or swe_vs_oracle_medium or full_size_swe_c3" -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 240 python -u bench.py --no-cold > $O/c3.json 2> $O/c3.err
timeout -k 10 240 python -u bench.py --no-cold > $O/c3b.json 2> $O/c3b.err
timeout -k 10 300 python -u tools/host_overhead.py 40 > $O/host.txt 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 6 --warmup 1 --no-cpu-baseline --no-cold > $O/prof.json 2> $O/prof.err
f=$(find $O/prof -name '*kernel_trace.csv' | head -n 1)
(cd tools && python trace_timeline.py ../$f 600) > $O/timeline.txt
echo host-done
