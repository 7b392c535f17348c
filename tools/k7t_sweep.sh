#!/bin/bash
# K7t schedule sweep: SPIS_K7T_CHUNK values under rocprofv3 kernel trace of the C3 bench
# (constraint_gram_sym_kernel mean per value in gpurun_out/k7t_<chunk>/run_kernel_stats.csv)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for ch in "$@"; do
  SPIS_K7T_CHUNK=$ch timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/k7t_$ch -o run \
    -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 2 > gpurun_out/k7t_$ch.log 2>&1 || exit 1
  python3 -c "
import csv,sys
for r in csv.DictReader(open('gpurun_out/k7t_$ch/run_kernel_stats.csv')):
    if 'gram_sym' in r['Name']: print('chunk $ch', r['Calls'], '%.1f us' % (float(r['AverageNs'])/1e3))
" || exit 1
  tail -c 300 gpurun_out/k7t_$ch.log | grep -o '"value": [0-9.]*' || true
done
