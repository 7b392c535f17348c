set -e
mkdir -p gpurun_out/r06lags
make tools/chainbench > gpurun_out/r06lags/build.log 2>&1
timeout -k 10 120 ./tools/chainbench 1002252 20 lags > gpurun_out/r06lags/lags.txt 2>&1
cat gpurun_out/r06lags/lags.txt
