set -e
mkdir -p gpurun_out/r06ph
make phases > gpurun_out/r06ph/build.log 2>&1
SPIS_LIBRARY=tools/libspis_phases.so timeout -k 10 300 python tools/host_phases.py 60 > gpurun_out/r06ph/phases.txt 2>&1
cat gpurun_out/r06ph/phases.txt | tail -45
