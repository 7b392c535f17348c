"""Summarise tools/gc_sweep.sh output: per run, the rel errors and the Gram kernel durations."""
import csv
import glob
import os
import sys

for d in sorted(glob.glob(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/gs_*")):
    if not os.path.isdir(d):
        continue
    print(os.path.basename(d))
    log = d + ".log"
    if os.path.exists(log):
        for line in open(log):
            if "rel err" in line:
                print("   ", line.rstrip())
    out = {}
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        n = r["Kernel_Name"]
        if "constraint_gram" in n or "transpose" in n or "reduce" in n:
            out.setdefault(n.split("(")[0][-42:], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in out.items():
        print("   ", k, [round(x, 1) for x in v])
