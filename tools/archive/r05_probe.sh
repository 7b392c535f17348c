#!/bin/bash
# Round 5: SpMV gather-latency probe (kbench slab: the solver's dual kernel vs the same kernel
# with its x gathers replaced by coalesced / broadcast loads), C3 and C5 matrices.
set -e
O=${1:-gpurun_out/r05probe}
mkdir -p "$O"
timeout -k 10 300 python tools/dump_matrix.py 289 /tmp/kbench_mat > $O/dump3.txt 2>&1
timeout -k 10 200 ./tools/kbench /tmp/kbench_mat slab > $O/slab_c3.txt 2>&1
timeout -k 10 600 python tools/dump_matrix.py 913 /tmp/kbench_mat5 > $O/dump5.txt 2>&1
timeout -k 10 300 ./tools/kbench /tmp/kbench_mat5 slab > $O/slab_c5.txt 2>&1

cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in "--method cgmres_p --steps 4" "--tol 1e-7 --steps 6"; do
  tag=$(echo $m | tr -d ' -' | cut -c1-16)
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$tag -o run -- python3 -u bench.py $m --warmup 1 --no-cpu-baseline --no-cold > $O/$tag.json 2> $O/$tag.err
  f=$(find $O/prof_$tag -name '*kernel_trace.csv' | head -n 1); cp "$f" $O/trace_$tag.csv
  (cd tools && python trace_timeline.py ../$O/trace_$tag.csv 600) > $O/timeline_$tag.txt
done
echo traces-done
