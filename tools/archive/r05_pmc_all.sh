#!/bin/bash
# Round 5: PMC traffic files at HEAD for C3, C2, C4, C5 (tools/r05_pmc.sh per configuration).
set -e
for c in c3 c2 c4 c5; do
  bash tools/r05_pmc.sh $c > gpurun_out/pmc_$c.log 2>&1
done
echo pmc-all-done
