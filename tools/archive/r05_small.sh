#!/bin/bash
# Round 5: K2s publishes the previous residual first; coalesced K7t / K7m / linear-term reductions.
# Tests, then C2 / C4 / C3 benches and C2 / C4 timelines.
O=${1:-gpurun_out/r05small2}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -k "k2s or golden or constraint_terms or k7t or incremental or c4 or lkdv" -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stop"; exit $rc; fi
set -e
for c in c2 c4 c3; do
  timeout -k 10 240 python -u bench.py --config $c --no-cold --no-cpu-baseline > $O/$c.json 2> $O/$c.err
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in c2 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$c -o run -- python3 -u bench.py --config $c --steps 6 --warmup 1 --no-cpu-baseline --no-cold > $O/p$c.json 2> $O/p$c.err
  f=$(find $O/prof_$c -name '*kernel_trace.csv' | head -n 1)
  (cd tools && python trace_timeline.py ../$f 600) > $O/timeline_$c.txt
done
echo small2-done
