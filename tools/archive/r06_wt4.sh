# K2s's q_{j+1} stored write-through (SPIS_STORE_WT bit 16) at C4 and C2
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06wt4
mkdir -p $o
timeout -k 10 300 env SPIS_STORE_WT=17 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "k2s or golden or full_size_lkdv_c2" > $o/tests.log 2>&1
tail -2 $o/tests.log
for cfg in c4 c2; do
for r in 1 2 3; do
for wt in 17 1; do
timeout -k 10 300 env SPIS_STORE_WT=$wt python -u bench.py --config $cfg --steps 50 --warmup 5 --no-cpu-baseline --no-cold > $o/${cfg}_${wt}_$r.json 2> $o/${cfg}_${wt}_$r.err
python -c "import json;d=json.load(open('$o/${cfg}_${wt}_$r.json'));k=d['kernels'];print('$cfg wt=$wt', round(d['value']), round(k['mgs_chain_us_mean'],2), round(k['spmv_dual_us'],2))"
done
done
done
