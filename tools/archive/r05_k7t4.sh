#!/bin/bash
# Round 5: K7t at 4 waves per SIMD (128 VGPRs, grid 1,024): constraint tests, C3 bench and stats.
set -e
O=${1:-gpurun_out/r05k7t4}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "bit_identical or constraint or incremental or golden or full_size_swe_c3 or k7t or c5_cycle0" -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || true
timeout -k 10 240 python -u bench.py --no-cold --no-cpu-baseline > $O/c3.json 2> $O/c3.err
timeout -k 10 240 python -u bench.py --no-cold --no-cpu-baseline > $O/c3b.json 2> $O/c3b.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cold > $O/prof.json 2> $O/prof.err
echo k7t4-done
