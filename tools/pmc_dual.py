"""HBM bytes per launch of the fused dual SpMV from separate rocprofv3 --pmc FETCH_SIZE /
WRITE_SIZE passes (MI355X_MICROARCH.md's recipe): the calibration streams of `tools/kbench <dir>
pmc` give the unit correction (FETCH_SIZE reports half of the bytes read by 8-B and 4-B per-lane
streams on gfx950; WRITE_SIZE is exact).  Writes profiles/spmv_dual_traffic.json.

usage: python tools/pmc_dual.py FETCH.csv WRITE.csv [out.json] [--kernel NAME]
           [--calib CAL_FETCH.csv CAL_WRITE.csv] [--source TEXT]
FETCH/WRITE are the kernel's passes (kbench pmc mode, or the bench itself); without --calib the
calibration kernels are taken from the same files."""
import csv
import json
import statistics
import sys

N, NNZ = 1002252, 12528150
ALG = 12 * NNZ + 4 * (N + 1) + 32 * N
GIB_KB = 1 << 20


def rows(path):
    return list(csv.DictReader(open(path)))


def mean_kb(rs, name_part, counter, sel=slice(None)):
    rs = sorted(rs, key=lambda r: int(r["Dispatch_Id"]))
    v = [float(r["Counter_Value"]) for r in rs if name_part in r["Kernel_Name"] and r["Counter_Name"] == counter][sel]
    return statistics.mean(v), len(v)


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("out", nargs="?", default="profiles/spmv_dual_traffic.json")
    ap.add_argument("--kernel", default="spmv_pipe_kernel<1024, 4")
    ap.add_argument("--calib", nargs=2, default=None)
    ap.add_argument("--source", default="separate rocprofv3 --pmc passes of tools/kbench pmc mode")
    ap.add_argument("--launches", default=None, help="python slice of the kernel's launches, e.g. 5: (cold ones)")
    a = ap.parse_args()
    f, w = rows(a.fetch), rows(a.write)
    out = a.out
    cf, cw = (rows(a.calib[0]), rows(a.calib[1])) if a.calib else (f, w)
    cal8, _ = mean_kb(cf, "calib_read8", "FETCH_SIZE")
    calw, _ = mean_kb(cw, "calib_write8", "WRITE_SIZE")
    fetch_corr = GIB_KB / cal8   # ~2 on gfx950
    write_corr = GIB_KB / calw   # ~1
    sel = slice(*[int(t) if t else None for t in a.launches.split(":")]) if a.launches else slice(None)
    fk, nf = mean_kb(f, a.kernel, "FETCH_SIZE", sel)
    wk, nw = mean_kb(w, a.kernel, "WRITE_SIZE", sel)
    rd = fk * 1024 * fetch_corr
    wr = wk * 1024 * write_corr
    res = {
        "kernel": f"{a.kernel} (true-residual SpMV of x_j fused with the Arnoldi SpMV of z_{{j+2}}), "
                  "swe C3 N=1,002,252 nnz=12,528,150",
        "source": f"{a.fetch}, {a.write} ({a.source}; {nf} / {nw} launches)",
        "calibration": f"same passes: 1 GiB read8 -> FETCH_SIZE {cal8:.0f} KB (x{fetch_corr:.3f}); "
                       f"1 GiB write8 -> WRITE_SIZE {calw:.0f} KB (x{write_corr:.3f})",
        "fetch_size_kb_raw": fk,
        "write_size_kb_raw": wk,
        "read_bytes_per_launch": rd,
        "write_bytes_per_launch": wr,
        "bytes_per_launch": rd + wr,
        "algorithmic_bytes_per_launch": ALG,
        "note": "reads exceed the algorithmic bytes mainly through x_j and z gathered by several XCD L2s",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
