"""HBM bytes per launch of the fused dual SpMV from separate rocprofv3 --pmc FETCH_SIZE /
WRITE_SIZE passes of `tools/kbench <dir> pmc` (MI355X_MICROARCH.md's recipe): the calibration
streams in the same passes give the unit correction (FETCH_SIZE reports half of the bytes read by
8-B and 4-B per-lane streams on gfx950; WRITE_SIZE is exact).  Writes profiles/spmv_dual_traffic.json.

usage: python tools/pmc_dual.py FETCH.csv WRITE.csv [out.json]"""
import csv
import json
import statistics
import sys

N, NNZ = 1002252, 12528150
ALG = 12 * NNZ + 4 * (N + 1) + 32 * N
GIB_KB = 1 << 20


def rows(path):
    return list(csv.DictReader(open(path)))


def mean_kb(rs, name_part, counter):
    v = [float(r["Counter_Value"]) for r in rs if name_part in r["Kernel_Name"] and r["Counter_Name"] == counter]
    return statistics.mean(v), len(v)


def main():
    f, w = rows(sys.argv[1]), rows(sys.argv[2])
    out = sys.argv[3] if len(sys.argv) > 3 else "profiles/spmv_dual_traffic.json"
    cal8, _ = mean_kb(f, "calib_read8", "FETCH_SIZE")
    calw, _ = mean_kb(w, "calib_write8", "WRITE_SIZE")
    fetch_corr = GIB_KB / cal8   # ~2 on gfx950
    write_corr = GIB_KB / calw   # ~1
    fk, nf = mean_kb(f, "spmv_dual_kernel<1024, 0>", "FETCH_SIZE")
    wk, nw = mean_kb(w, "spmv_dual_kernel<1024, 0>", "WRITE_SIZE")
    rd = fk * 1024 * fetch_corr
    wr = wk * 1024 * write_corr
    res = {
        "kernel": "spmv_dual_kernel<1024> (true-residual SpMV of x_j fused with the Arnoldi SpMV of z_{j+2}), "
                  "swe C3 N=1,002,252 nnz=12,528,150",
        "source": f"{sys.argv[1]}, {sys.argv[2]} (separate rocprofv3 --pmc passes of tools/kbench pmc mode, "
                  f"solver's kDualCap row blocks; {nf} / {nw} launches)",
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
