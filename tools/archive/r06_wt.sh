# write-through output stores A/B (SPIS_STORE_WT), the start-up host phases, the parity subset
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06wt
mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "golden or bit_identical or bit_exact or chain_matches or full_size_swe_vs_oracle or first_chain" > $o/tests.log 2>&1
tail -2 $o/tests.log
for r in 1 2 3; do
for wt in 1 0; do
timeout -k 10 300 env SPIS_STORE_WT=$wt python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-cold --no-wrapper > $o/c3_${wt}_$r.json 2> $o/c3_${wt}_$r.err
python -c "import json;d=json.load(open('$o/c3_${wt}_$r.json'));k=d['kernels'];print('wt=$wt', round(d['value']), round(k['mgs_chain_us_mean'],2), round(k['spmv_dual_us'],2), round(k['spmv_arnoldi_us'],2), round(k['gemv_us_mean'],2))"
done
done
for it in 0 1 2 10; do
timeout -k 10 300 env SPIS_LIBRARY=tools/libspis_phases.so SPIS_PHASE_ITER=$it python -u tools/host_phases.py 80 > $o/phases_$it.txt 2>&1
grep -E "start-up|iteration" $o/phases_$it.txt
done
