#!/bin/bash
# A/B of bench options, interleaved: tools/ab_bench.sh ROUNDS "opts A" "opts B" ...
# ("-" = no options); prints it/s and the dual / chain kernel means per run.
set -e
rounds=$1; shift
for r in $(seq 1 "$rounds"); do
  for opt in "$@"; do
    o=$opt; [ "$o" = - ] && o=""
    v=$(timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 3 $o | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); k=d['kernels']; print('%.0f it/s dual %.1f chain %.1f arnoldi %.1f' % (d['value'], k['spmv_dual_us'], k['mgs_chain_us_mean'], k['spmv_arnoldi_us']))")
    echo "round $r [$opt]: $v"
  done
done
