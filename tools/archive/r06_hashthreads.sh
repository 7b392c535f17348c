# drop-in wrapper rate against the verifier's thread count (SPIS_HASH_THREADS), two runs each
set -e
o=gpurun_out/r06ht
mkdir -p $o
for t in 16 12 8 16 12 8; do
timeout -k 10 300 env SPIS_HASH_THREADS=$t python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-cold > $o/c3_$t.json 2> $o/c3_$t.err
python -c "import json;d=json.load(open('$o/c3_$t.json'));w=d['wrapper'];print($t, round(d['value']), round(w['value']), round(w['frac_of_value'],3), round(w['ms_per_call'],3), round(w['verify_ms'],2), {k: round(v,3) for k,v in w['phases_ms'].items()})"
done
