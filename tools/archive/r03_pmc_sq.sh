#!/bin/bash
# C5 SpMV stall profile: the counter list of this GPU, then SQ wave-state counters of the
# standalone Arnoldi / dual SpMV launches (tools/spmv_pmc.py), one pass under its own kill limit
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${1:-gpurun_out/pmcsq}
mkdir -p "$O"
timeout -s KILL 60 rocprofv3 -L > "$O/avail.txt" 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
  --output-format csv -d "$O/sq" -o run -- python tools/spmv_pmc.py 913 0 1 1 > "$O/sq.log" 2>&1
echo done
