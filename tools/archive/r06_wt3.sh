# write-through stores in K2w's update pass (SPIS_STORE_WT bit 1) at C5 and on the one-rank distributed path
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06wt3
mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "golden or self_halo or k2w or chain_matches or restarted" > $o/tests.log 2>&1
tail -2 $o/tests.log
for wt in 1 0 1 0; do
timeout -k 10 300 env SPIS_STORE_WT=$wt python -u bench.py --force-distributed --steps 20 --no-cpu-baseline > $o/d1_${wt}.json 2> $o/d1_${wt}.err
python -c "import json;d=json.load(open('$o/d1_${wt}.json'));k=d['kernels'];print('dist1 wt=$wt', round(d['value']), round(k['mgs_us_mean'],2), round(k['spmv_us'],2))"
done
for wt in 1 0; do
timeout -k 10 500 env SPIS_STORE_WT=$wt python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-cold > $o/c5_${wt}.json 2> $o/c5_${wt}.err
python -c "import json;d=json.load(open('$o/c5_${wt}.json'));k=d['kernels'];print('c5 wt=$wt', round(d['value'],1), round(k['mgs_chain_us_mean'],1), round(k['spmv_dual_us'],1))"
done
