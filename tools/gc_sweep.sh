#!/bin/bash
# tuning sweep of the constraint-Gram kernels (tools/gram_check.py under rocprofv3 kernel trace)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {  # name, env..., then M p
  local name=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$name -o run -- python3 tools/gram_check.py $M $P > gpurun_out/$name.log 2>&1
}
M=40 P=30 run gs_small8 SPIS_GRAM_GRID=8 || exit 1
M=289 P=30 run gs_c3 SPIS_X=0 || exit 1
