set -e
mkdir -p gpurun_out/r06bar
make tools/chainbench > gpurun_out/r06bar/build.log 2>&1
timeout -k 10 120 ./tools/chainbench 1002252 20 trace > gpurun_out/r06bar/trace.txt 2>&1
grep event gpurun_out/r06bar/trace.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "golden or chain or first_chain" > gpurun_out/r06bar/tests.log 2>&1
tail -1 gpurun_out/r06bar/tests.log
for r in 1 2; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-cold --no-wrapper > gpurun_out/r06bar/c3_$r.json 2> gpurun_out/r06bar/c3_$r.err
python -c "import json;d=json.load(open('gpurun_out/r06bar/c3_$r.json'));print(d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done
