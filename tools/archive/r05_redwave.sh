#!/bin/bash
# Round 5: column reductions one wave per output: bitwise A/B tests, constraint tests, C3/C2 benches, C3 stats.
set -e
O=${1:-gpurun_out/r05rw}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "bit_identical or constraint or incremental or golden or full_size_swe_c3 or k7t" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 240 python -u bench.py --no-cold --no-cpu-baseline > $O/c3.json 2> $O/c3.err
timeout -k 10 240 python -u bench.py --config c2 --no-cold --no-cpu-baseline > $O/c2.json 2> $O/c2.err
SPIS_REDUCE_WAVE=0 timeout -k 10 240 python -u bench.py --config c2 --no-cold --no-cpu-baseline > $O/c2_off.json 2> $O/c2_off.err
timeout -k 10 240 python -u bench.py --config c2 --no-cold --no-cpu-baseline > $O/c2b.json 2> $O/c2b.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold > $O/prof.json 2> $O/prof.err
echo rw-done
