set -e
mkdir -p gpurun_out/r06perm
timeout -k 10 300 python -u tools/perm_ab.py 289 20 > gpurun_out/r06perm/c3.log 2>&1
cat gpurun_out/r06perm/c3.log | tail -3
