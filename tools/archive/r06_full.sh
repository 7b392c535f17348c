# full GPU suite, smoke, the C3 line and the K2q phase trace (one box)
set -e
mkdir -p gpurun_out/r06full
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/r06full/tests.log 2>&1
tail -3 gpurun_out/r06full/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06full/smoke.log 2>&1
tail -1 gpurun_out/r06full/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06full/c3.json 2> gpurun_out/r06full/c3.err
python -c "import json;d=json.load(open('gpurun_out/r06full/c3.json'));print(d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['wrapper']['value'], d['wrapper']['frac_of_value'], d['wrapper']['phases_ms'])"
make tools/chainbench > gpurun_out/r06full/cb_build.log 2>&1
timeout -k 10 120 ./tools/chainbench 1002252 20 trace > gpurun_out/r06full/trace.txt 2>&1
grep "event" gpurun_out/r06full/trace.txt
