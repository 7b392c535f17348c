"""Kernel statistics CSV (the columns of `rocprofv3 --stats`' kernel_stats.csv) from a rocprofv3
rocpd SQLite database, for runs where rocprofv3 wrote only `<name>_results.db`.

usage: python tools/rocpd_stats.py gpurun_out/prof/r02e_results.db profiles/r02e_bench_kernel_stats.csv
"""
import csv
import sqlite3
import statistics
import sys
from collections import defaultdict


def main(db, out):
    con = sqlite3.connect(db)
    durs = defaultdict(list)
    for name, dur in con.execute("select name, duration from kernels"):
        durs[name].append(int(dur))
    total = sum(sum(v) for v in durs.values())
    rows = sorted(durs.items(), key=lambda kv: -sum(kv[1]))
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        for name, v in rows:
            s = sum(v)
            w.writerow([name, len(v), s, s / len(v), round(100.0 * s / total, 2), min(v), max(v),
                        statistics.pstdev(v) if len(v) > 1 else 0.0])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
