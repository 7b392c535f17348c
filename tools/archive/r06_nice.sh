# drop-in wrapper rate with the verifier's digest threads at a lower priority (SPIS_HASH_NICE) or not
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06nice
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_host_caches.py -m gpu -k "in_place or cached_constraint_vector or pinned" > $o/tests.log 2>&1
tail -2 $o/tests.log
for r in 1 2 3; do
for nice in 10 0; do
timeout -k 10 300 env SPIS_HASH_NICE=$nice python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-cold > $o/c3_${nice}_$r.json 2> $o/c3_${nice}_$r.err
python -c "import json;d=json.load(open('$o/c3_${nice}_$r.json'));w=d['wrapper'];print('nice=$nice', round(d['value']), round(w['value']), round(w['frac_of_value'],3), round(w['ms_per_call'],3), round(w['verify_ms'],2), {k: round(v,3) for k,v in w['phases_ms'].items()})"
done
done
