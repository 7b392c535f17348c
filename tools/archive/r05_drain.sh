#!/bin/bash
# Round 5: no end-of-solve event wait when the last residual came from the last kernel: host phases,
# C3/C4/C2 benches, the whole GPU suite.
set -e
O=${1:-gpurun_out/r05drain}
mkdir -p "$O"
SPIS_LIBRARY=tools/libspis_phases.so timeout -k 10 300 python -u tools/host_phases.py 80 > $O/phases.txt 2>&1
timeout -k 10 240 python -u bench.py --no-cold --no-cpu-baseline > $O/c3.json 2> $O/c3.err
timeout -k 10 240 python -u bench.py --no-cold --no-cpu-baseline > $O/c3b.json 2> $O/c3b.err
timeout -k 10 240 python -u bench.py --config c4 --no-cold --no-cpu-baseline > $O/c4.json 2> $O/c4.err
timeout -k 10 240 python -u bench.py --config c2 --no-cold --no-cpu-baseline > $O/c2.json 2> $O/c2.err
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/gputest.log 2>&1
echo drain-done
