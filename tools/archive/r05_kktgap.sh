#!/bin/bash
set -e
O=gpurun_out/r05kkt
mkdir -p $O
timeout -k 10 300 python -u tools/kkt_gap.py 30 > $O/kkt.txt 2>&1
echo kkt-done
