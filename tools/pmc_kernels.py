"""HBM bytes per launch of every kernel of a bench run, from two separate rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE) over the same command.  The unit corrections (FETCH_SIZE x2 on gfx950,
WRITE_SIZE exact) come from the calibration streams of an earlier kbench pass (tools/pmc_dual.sh),
as MI355X_MICROARCH.md's HBM recipe prescribes.

usage: python tools/pmc_kernels.py FETCH.csv WRITE.csv CAL_FETCH.csv CAL_WRITE.csv out.json
"""
import collections
import csv
import json
import statistics
import sys


def per_kernel(path, counter):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            d[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return d


def calib(path, name, counter):
    return statistics.mean(float(r["Counter_Value"]) for r in csv.DictReader(open(path))
                           if name in r["Kernel_Name"] and r["Counter_Name"] == counter)


def main(fetch, write, cal_f, cal_w, out):
    fc = (1 << 20) / calib(cal_f, "calib_read8", "FETCH_SIZE")
    wc = (1 << 20) / calib(cal_w, "calib_write8", "WRITE_SIZE")
    f, w = per_kernel(fetch, "FETCH_SIZE"), per_kernel(write, "WRITE_SIZE")
    rows = []
    for k in sorted(f, key=lambda k: -sum(f[k])):
        rd = statistics.mean(f[k]) * 1024 * fc
        wr = statistics.mean(w[k]) * 1024 * wc if w.get(k) else 0.0
        rows.append({"kernel": k, "launches": len(f[k]), "read_MB": round(rd / 1e6, 1),
                     "write_MB": round(wr / 1e6, 1), "total_MB": round((rd + wr) / 1e6, 1)})
    res = {"source": f"{fetch}, {write}", "fetch_corr": fc, "write_corr": wc, "kernels": rows}
    json.dump(res, open(out, "w"), indent=1)
    for r in rows:
        print(f"{r['kernel'][:70]:70s} {r['launches']:4d} {r['read_MB']:8.1f} {r['write_MB']:8.1f}")


if __name__ == "__main__":
    main(*sys.argv[1:6])
