#!/bin/bash
# Round 5: K2q exchange-ahead (CW) debug: bitwise verify against the vmcnt(0) build, then shapes
# at three poll sleeps.
set -e
O=${1:-gpurun_out/r05cwd}
mkdir -p "$O"
timeout -k 10 120 ./tools/chainbench 1002252 20 verify > $O/verify.txt 2>&1 || true
timeout -k 10 120 ./tools/chainbench 1002252 20 ring > $O/ring1.txt 2>&1
timeout -k 10 120 ./tools/chainbench_s4 1002252 20 ring > $O/ring4.txt 2>&1
timeout -k 10 120 ./tools/chainbench_s16 1002252 20 ring > $O/ring16.txt 2>&1
echo dbg-done
