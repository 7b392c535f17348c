#!/bin/bash
# Round 5: bench warm-up reaches the two-workspace steady state; host phases of the last iteration.
set -e
O=${1:-gpurun_out/r05warm}
mkdir -p "$O"
SPIS_LIBRARY=tools/libspis_phases.so timeout -k 10 300 python -u tools/host_phases.py 80 > $O/phases.txt 2>&1
for i in 1 2; do timeout -k 10 240 python -u bench.py --no-cold --no-cpu-baseline > $O/c3_$i.json 2> $O/c3_$i.err; done
timeout -k 10 240 python -u bench.py --config c4 --no-cold --no-cpu-baseline > $O/c4.json 2> $O/c4.err
timeout -k 10 240 python -u bench.py --config c2 --no-cold --no-cpu-baseline > $O/c2.json 2> $O/c2.err
timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cold --no-cpu-baseline > $O/c5.json 2> $O/c5.err
echo warm-done
