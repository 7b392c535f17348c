set -e
mkdir -p gpurun_out/r03v
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03v/gputest.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03v/smoke.log 2>&1
timeout -k 10 240 python -u bench.py > gpurun_out/r03v/bench.log 2>&1
timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 1 > gpurun_out/r03v/c5.log 2>&1
timeout -k 10 240 python -u bench.py --force-distributed > gpurun_out/r03v/dist1.log 2>&1
timeout -k 10 240 python -u bench.py --config c2 > gpurun_out/r03v/c2.log 2>&1
timeout -k 10 240 python -u bench.py --config c4 > gpurun_out/r03v/c4.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03v/prof -o run -- python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cold > gpurun_out/r03v/prof.log 2>&1
