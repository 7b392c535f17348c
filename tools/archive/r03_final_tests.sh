#!/bin/bash
# the driver's round-end GPU checks at HEAD: pytest -m gpu, then smoke()
set -e
O=${1:-gpurun_out/final}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gputest.log" 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
