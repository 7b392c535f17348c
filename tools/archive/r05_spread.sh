#!/bin/bash
# Round 5: run-to-run spread of the bench lines on one box (C3 x5, C2 x3, C4 x3).
set -e
O=${1:-gpurun_out/r05sp}
mkdir -p "$O"
for i in 1 2 3 4 5; do
  timeout -k 10 240 python -u bench.py --no-cold --no-cpu-baseline > $O/c3_$i.json 2> $O/c3_$i.err
done
for c in c2 c4; do for i in 1 2 3; do
  timeout -k 10 240 python -u bench.py --config $c --no-cold --no-cpu-baseline > $O/${c}_$i.json 2> $O/${c}_$i.err
done; done
python - <<'PY' > $O/summary.txt
import json, glob, statistics
for c in ("c3", "c2", "c4"):
    v = [json.load(open(f))["value"] for f in sorted(glob.glob("gpurun_out/r05sp/%s_*.json" % c))]
    print(c, "runs", [round(x) for x in v], "median", round(statistics.median(v)), "min", round(min(v)), "max", round(max(v)))
PY
echo spread-done
