#!/bin/bash
# Round-5 validation on one GPU box (one gpurun call): pytest -m gpu (with the multi-rank solves),
# smoke(), every configuration's bench line (C3 also at tol 1e-7 and through cgmres_p), then
# rocprofv3 --kernel-trace --stats summaries of the C3 and C5 benches (csv) and a C3 kernel trace
# timeline.  Each GPU step has its own time limit; set -e ends the script at the first failure.
set -e
O=${1:-gpurun_out/r05v}
mkdir -p "$O"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > $O/gputest.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 240 python -u bench.py > $O/c3.json 2> $O/c3.err
timeout -k 10 240 python -u bench.py --tol 1e-7 > $O/c3_tol7.json 2> $O/c3_tol7.err
timeout -k 10 240 python -u bench.py --method cgmres_p > $O/c3_p.json 2> $O/c3_p.err
timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 1 > $O/c5.json 2> $O/c5.err
timeout -k 10 240 python -u bench.py --force-distributed > $O/dist1.json 2> $O/dist1.err
timeout -k 10 240 python -u bench.py --config c2 > $O/c2.json 2> $O/c2.err
timeout -k 10 240 python -u bench.py --config c4 > $O/c4.json 2> $O/c4.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_c3.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_c5.log 2>&1
f=$(find $O/prof_c3 -name '*kernel_trace.csv' | head -n 1)
(cd tools && python trace_timeline.py ../$f 600) > $O/timeline_c3.txt
echo validate-done
