# write-through store mask A/B (SPIS_STORE_WT: 1 MGS, 2 SpMV, 4 transpose/GEMV/copy) at C3, C4, C2
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06wt2
mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "golden or bit_identical or bit_exact or chain_matches or full_size_swe_vs_oracle or first_chain or k2s or incremental or constraint_terms" > $o/tests.log 2>&1
tail -2 $o/tests.log
for r in 1 2; do
for wt in 7 5 1 0; do
timeout -k 10 300 env SPIS_STORE_WT=$wt python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-cold --no-wrapper > $o/c3_${wt}_$r.json 2> $o/c3_${wt}_$r.err
python -c "import json;d=json.load(open('$o/c3_${wt}_$r.json'));k=d['kernels'];print('c3 wt=$wt', round(d['value']), round(k['mgs_chain_us_mean'],2), round(k['spmv_dual_us'],2), round(k['spmv_arnoldi_us'],2), round(k['gemv_us_mean'],2))"
done
done
for cfg in c4 c2; do
for wt in 7 0 7 0; do
timeout -k 10 300 env SPIS_STORE_WT=$wt python -u bench.py --config $cfg --steps 50 --warmup 5 --no-cpu-baseline --no-cold > $o/${cfg}_${wt}.json 2> $o/${cfg}_${wt}.err
python -c "import json;d=json.load(open('$o/${cfg}_${wt}.json'));k=d['kernels'];print('$cfg wt=$wt', round(d['value']), round(k['mgs_chain_us_mean'],2), round(k['spmv_dual_us'],2))"
done
done
