#!/bin/bash
# Round 5: K7t's transpose with the next tile in flight: bitwise A/B test, constraint tests, C3 A/B, C5.
set -e
O=${1:-gpurun_out/r05tp}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "pipelined_transpose or constraint or incremental or golden or full_size_swe_c3" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 240 python -u bench.py --no-cold --no-cpu-baseline > $O/c3.json 2> $O/c3.err
SPIS_TRANSPOSE_PIPE=0 timeout -k 10 240 python -u bench.py --no-cold --no-cpu-baseline > $O/c3_off.json 2> $O/c3_off.err
timeout -k 10 240 python -u bench.py --no-cold --no-cpu-baseline > $O/c3b.json 2> $O/c3b.err
timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cold --no-cpu-baseline > $O/c5.json 2> $O/c5.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold > $O/prof.json 2> $O/prof.err
echo tp-done
