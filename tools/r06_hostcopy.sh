#!/bin/bash
# A/B of the host copy / zero-scan piece size (tools/r06_hostcopy.py); host-only, run on the GPU box
set -e
mkdir -p gpurun_out/hc
for s in 16 20; do
  g++ -O3 -std=c++17 -fPIC -shared -I include -DSPIS_FINE_SHIFT=$s \
      structurepreservingiterativesolvers_amd/csrc/hash.cpp -o gpurun_out/hc/libhash_$s.so -lpthread
done
timeout -k 10 240 python3 -u tools/r06_hostcopy.py gpurun_out/hc/libhash_16.so \
    gpurun_out/hc/libhash_20.so 2>&1 | tee gpurun_out/hc/hostcopy.txt
