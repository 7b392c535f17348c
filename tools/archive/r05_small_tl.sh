#!/bin/bash
# Round 5: C2 and C4 kernel-trace timelines (gaps between kernels at small N).
set -e
O=${1:-gpurun_out/r05stl}
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in c2 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$c -o run -- python3 -u bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline --no-cold > $O/$c.json 2> $O/$c.err
  f=$(find $O/prof_$c -name '*kernel_trace.csv' | head -n 1)
  (cd tools && python trace_timeline.py ../$f 600) > $O/timeline_$c.txt
done
echo stl-done
