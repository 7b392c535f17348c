#!/bin/bash
# Round 5: K2s16 (1,024-thread workgroups, four resident chunks + one streamed) at C4's N.
set -e
O=${1:-gpurun_out/r05k16}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "k2s_onepass" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/k2s.log 2>&1
timeout -k 10 240 python -u bench.py --config c4 --no-cold --no-cpu-baseline > $O/c4.json 2> $O/c4.err
SPIS_K2S16=0 timeout -k 10 240 python -u bench.py --config c4 --no-cold --no-cpu-baseline > $O/c4_off.json 2> $O/c4_off.err
timeout -k 10 240 python -u bench.py --config c4 --no-cold --no-cpu-baseline > $O/c4b.json 2> $O/c4b.err
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "lkdvrk or golden or lkdv" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline --no-cold > $O/prof.json 2> $O/prof.err
echo k16-done
