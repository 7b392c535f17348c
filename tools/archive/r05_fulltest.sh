#!/bin/bash
# Round 5: the whole GPU suite at HEAD, then smoke().
set -e
O=${1:-gpurun_out/r05ft}
mkdir -p "$O"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > $O/gputest.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo fulltest-done
