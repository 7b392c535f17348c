set -e
mkdir -p gpurun_out/r06wrap
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "in_place or cached_constraint_vector or golden or x0_zero or incremental_constraint or pipelined_transpose" -m gpu > gpurun_out/r06wrap/tests.log 2>&1
tail -3 gpurun_out/r06wrap/tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-cold > gpurun_out/r06wrap/c3.json 2> gpurun_out/r06wrap/c3.err
python -c "import json;d=json.load(open('gpurun_out/r06wrap/c3.json'));print(d['value']);print(json.dumps(d['wrapper'],indent=1))"
