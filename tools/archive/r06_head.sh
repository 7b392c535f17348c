# HEAD check on one box: full GPU suite, smoke, the C3 line, and a kernel trace of the C3 bench
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06head
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > $o/tests.log 2>&1
tail -3 $o/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
tail -1 $o/smoke.log
timeout -k 10 300 python -u bench.py > $o/c3.json 2> $o/c3.err
python -c "import json;d=json.load(open('$o/c3.json'));print(d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['wrapper']['value'], d['wrapper']['frac_of_value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-wrapper --no-cold > $o/prof_bench.json 2> $o/prof_bench.err
echo "rocprof done"
bash tools/r06_hashthreads.sh
