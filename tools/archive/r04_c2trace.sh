#!/bin/bash
# C2 kernel traces: the default (K2w at small N) and K2q forced, per-solve busy time and gaps
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${1:-gpurun_out/r04c2t}
mkdir -p $O
for sm in 225000 0; do
  SPIS_K2W_SMALL_N=$sm timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/p$sm -o run -- python3 -u bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline --no-cold > $O/c2_$sm.json 2> $O/c2_$sm.err
  f=$(find $O/p$sm -name '*kernel_trace.csv' | head -n 1); cp "$f" $O/trace_$sm.csv
  python tools/trace_gaps.py $O/trace_$sm.csv > $O/gaps_$sm.txt
done
