set -e
O=${1:-gpurun_out/r03v}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 240 python -u bench.py > $O/bench.log 2>&1
timeout -k 10 240 python -u bench.py --col16 2 --no-cpu-baseline > $O/bench_c16.log 2>&1
timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 1 > $O/c5.log 2>&1
timeout -k 10 240 python -u bench.py --force-distributed > $O/dist1.log 2>&1
timeout -k 10 240 python -u bench.py --config c2 > $O/c2.log 2>&1
timeout -k 10 240 python -u bench.py --config c4 > $O/c4.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold > $O/prof.log 2>&1
