set -e
mkdir -p gpurun_out/r06pref
make tools/chainbench > gpurun_out/r06pref/build.log 2>&1
timeout -k 10 120 ./tools/chainbench 1002252 20 lags > gpurun_out/r06pref/lags.txt 2>&1
cat gpurun_out/r06pref/lags.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "golden or chain or first_chain" > gpurun_out/r06pref/tests.log 2>&1
tail -2 gpurun_out/r06pref/tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-cold --no-wrapper > gpurun_out/r06pref/c3.json 2> gpurun_out/r06pref/c3.err
python -c "import json;d=json.load(open('gpurun_out/r06pref/c3.json'));print(d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
