set -e
mkdir -p gpurun_out/r06wrap2
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_host_caches.py -k "in_place or cached_constraint_vector or golden or pinned or x0_zero or first_chain" -m gpu > gpurun_out/r06wrap2/tests.log 2>&1
tail -2 gpurun_out/r06wrap2/tests.log
for r in 1 2; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-cold > gpurun_out/r06wrap2/c3_$r.json 2> gpurun_out/r06wrap2/c3_$r.err
python -c "import json;d=json.load(open('gpurun_out/r06wrap2/c3_$r.json'));w=d['wrapper'];print(round(d['value']), round(w['value']), round(w['frac_of_value'],3), round(w['ms_per_call'],3), round(w['verify_ms'],2), {k: round(v,3) for k,v in w['phases_ms'].items()})"
done
