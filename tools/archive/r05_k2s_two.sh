#!/bin/bash
# Round 5: K2s two-chunk mode at C2 (SPIS_K2S_TWO_MIN A/B): fewer workgroups in the hand-offs.
set -e
O=${1:-gpurun_out/r05two}
mkdir -p "$O"
for t in 4096 256 4096 256 128; do
  SPIS_K2S_TWO_MIN=$t timeout -k 10 240 python -u bench.py --config c2 --no-cold --no-cpu-baseline > $O/c2_$t.json 2> $O/c2_$t.err
  python -c "import json; d=json.load(open('$O/c2_$t.json')); print('two_min', $t, round(d['value']), d['kernels'].get('mgs_chain_us_mean'))" >> $O/summary.txt
done
SPIS_K2S_TWO_MIN=128 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "k2s_onepass or lkdv" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
echo two-done
