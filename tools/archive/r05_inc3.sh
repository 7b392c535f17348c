#!/bin/bash
# Round 5: constrained steps' increments on the main stream behind the chain, one K6i pass
# (SpMV + dots): tests, C3 tol 1e-7 / cgmres_p / default benches, kernel traces of the first two.
O=${1:-gpurun_out/r05inc3}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -k "incremental or golden or constraint_terms or restarted_cgmres or swe_vs_oracle_medium or cgmres_p or lkdvrk_gl3 or c5" -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stop"; exit $rc; fi
set -e
timeout -k 10 240 python -u bench.py --tol 1e-7 --steps 20 --no-cpu-baseline --no-cold > $O/c3_tol7.json 2> $O/c3_tol7.err
timeout -k 10 240 python -u bench.py --method cgmres_p --steps 10 --no-cpu-baseline --no-cold > $O/c3_p.json 2> $O/c3_p.err
timeout -k 10 240 python -u bench.py --steps 20 --no-cpu-baseline --no-cold > $O/c3.json 2> $O/c3.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in "--method cgmres_p --steps 4" "--tol 1e-7 --steps 6"; do
  tag=$(echo $m | tr -d ' -' | cut -c1-16)
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$tag -o run -- python3 -u bench.py $m --warmup 1 --no-cpu-baseline --no-cold > $O/$tag.json 2> $O/$tag.err
  f=$(find $O/prof_$tag -name '*kernel_trace.csv' | head -n 1); cp "$f" $O/trace_$tag.csv
  (cd tools && python trace_timeline.py ../$O/trace_$tag.csv 600) > $O/timeline_$tag.txt
done
echo inc3-done
