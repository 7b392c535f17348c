# K7t with pipelined gathers (SPIS_K7T_PIPE): bitwise test, then the C3 line and kernel stats A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06k7tp
mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "k7t or constraint_terms or incremental or pipelined_transpose" > $o/tests.log 2>&1
tail -3 $o/tests.log
for p in 1 0; do
SPIS_K7T_PIPE=$p timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof$p -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-wrapper --no-cold > $o/prof$p.json 2> $o/prof$p.err
python3 tools/rocpd_stats.py $o/prof$p/run_results.db $o/stats$p.csv
grep -i "constraint_gram" $o/stats$p.csv | cut -c1-60,200-
done
for r in 1 2; do
for p in 1 0; do
timeout -k 10 300 env SPIS_K7T_PIPE=$p python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-cold --no-wrapper > $o/c3_${p}_$r.json 2> $o/c3_${p}_$r.err
python -c "import json;d=json.load(open('$o/c3_${p}_$r.json'));print('c3 pipe=$p', round(d['value']))"
done
done
