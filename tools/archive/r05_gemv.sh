#!/bin/bash
# Round 5: the update GEMV with its basis loop unrolled by 8: golden/constraint tests, C3 bench, stats.
set -e
O=${1:-gpurun_out/r05gemv}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "golden or bit_identical or constraint or full_size_swe_c3 or gemv or iterate" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 240 python -u bench.py --no-cold --no-cpu-baseline > $O/c3.json 2> $O/c3.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold > $O/prof.json 2> $O/prof.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof5 -o run -- python3 -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-cold > $O/prof5.json 2> $O/prof5.err
echo gemv-done
