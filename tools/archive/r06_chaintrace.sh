set -e
mkdir -p gpurun_out/r06ct
make tools/chainbench > gpurun_out/r06ct/build.log 2>&1
timeout -k 10 120 ./tools/chainbench 1002252 20 trace > gpurun_out/r06ct/trace.txt 2>&1
timeout -k 10 120 ./tools/chainbench 1002252 20 > gpurun_out/r06ct/variants.txt 2>&1
head -40 gpurun_out/r06ct/trace.txt
