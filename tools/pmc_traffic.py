"""Per-launch HBM traffic of the bench's SpMV and MGS launches, with the provenance bench.py checks
before it reports the figures as ``roofline.traffic`` (bench.load_traffic).

GPU box, two separate rocprofv3 passes over the same short bench (MI355X_MICROARCH.md: one
counter group per pass), then the reduction (tools/archive/r04_pmc.sh runs all three):

  rocprofv3 --pmc FETCH_SIZE --output-format csv -d D/f -o run -- python tools/pmc_traffic.py run c3
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d D/w -o run -- python tools/pmc_traffic.py run c3
  python tools/pmc_traffic.py reduce c3 D/f/..._counter_collection.csv D/w/..._counter_collection.csv OUT.json

``run`` is ``bench.py --config CFG --steps 3 --warmup 1 --no-cpu-baseline --no-wrapper`` with the default
options.  Its last launches are the bench's standalone timing of the solver's SpMV
(spis_spmv_bench: 22 back to back, then 22 each behind a 1 GiB evicting read), which also carry the
calibration: the evicting read (stream_read_kernel, 1 GiB of 16-B loads per lane) gives
FETCH_SIZE's unit, the 1 GiB zero-fill of its buffer (__amd_rocclr_fillBufferAligned)
WRITE_SIZE's.  Reported per launch: the dual SpMV in the solver and standalone cold, the MGS of
one Arnoldi step (every kernel of it, mean over the chain positions the solves ran), the
constrained step's basis transpose and K7t / K7m Gram launches, with the SHA-256 of
csrc/kernels.hip and the options.
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import math
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)
BENCH_SPMV = 22  # spis_spmv_bench launches per (kind, cold): 2 untimed + 20 (bench.py)
MGS_KERNELS = ("mgs_chain_lag_kernel", "mgs_chain_big_kernel", "mgs_chain_kernel", "icwy_dot_kernel", "icwy_onepass_kernel",
               "cgs_finalize_kernel", "cgs_update_kernel", "normalize_kernel", "mgs_step_kernel")


def _rows(path, counter):
    """(dispatch id, kernel, value) of one counter, in dispatch order."""
    out = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            out.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    return sorted(out)


def reduce(cfg, fetch_csv, write_csv, out):
    sys.argv = ["bench.py"]
    import bench

    f, w = _rows(fetch_csv, "FETCH_SIZE"), _rows(write_csv, "WRITE_SIZE")
    cal_f = [v for _, k, v in f if "stream_read_kernel" in k]
    cal_w = [v for _, k, v in w if "fillBufferAligned" in k]
    if not cal_f or not cal_w:
        raise SystemExit("calibration launches missing from the counter files")
    fc = GIB / (statistics.median(cal_f) * 1024)  # counters in KiB
    # the calibration fill is the 1 GiB eviction memset; the solver's own workspace
    # memsets are fills too (2.4 GB at C5), so pick the launch nearest 1 GiB, not the max
    wcal = min(cal_w, key=lambda v: abs(math.log(max(v, 1.0) * 1024 / GIB)))
    wc = GIB / (wcal * 1024)
    wmap = {d: v for d, _, v in w}
    byte = {d: v * 1024 * fc + wmap.get(d, 0.0) * 1024 * wc for d, _, v in f}
    names = {d: k for d, k, _ in f}
    dual = [d for d, k, _ in f if "spmv_pipe_kernel<2048, 4" in k or "spmv_dual_kernel" in k]
    if len(dual) < 2 * BENCH_SPMV + 1:
        raise SystemExit(f"{len(dual)} dual SpMV launches: expected the solver's and the bench's 44")
    solver_dual, warm, cold = dual[:-2 * BENCH_SPMV], dual[-2 * BENCH_SPMV:-BENCH_SPMV], dual[-BENCH_SPMV:]
    end_solver = solver_dual[-1]
    mgs = [d for d in byte if d <= end_solver and any(m in names[d] for m in MGS_KERNELS)]
    # one Arnoldi step's MGS = its chain launch, or (K2w) its dot / coefficient / update / normalise
    # launches: the count of steps is the count of chain launches or of icwy_dot launches
    steps = sum(1 for d in mgs if "mgs_chain" in names[d] or "icwy_dot" in names[d] or "icwy_onepass" in names[d])
    # the normalise of r0 (one per solve, after the r0 SpMV, epilogue kEpiR0 = 3) is not MGS
    solves = sum(1 for d in byte if d <= end_solver and ("spmv_pipe_kernel<2048, 3" in names[d]
                                                         or "spmv_rowblock_kernel<3>" in names[d]))
    norms = [byte[d] for d in mgs if "normalize_kernel" in names[d]]
    mgs_bytes = sum(byte[d] for d in mgs) - (statistics.mean(norms) * solves if norms else 0.0)
    res = {
        "config": cfg,
        "kernels_sha256": bench.kernels_sha256(),
        "git_rev": subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True,
                                  text=True).stdout.strip() or None,
        "options": None,  # filled below from the bench's own defaults
        "fetch_unit_correction": fc,
        "write_unit_correction": wc,
        "launches": {"dual_solver": len(solver_dual), "dual_warm": len(warm) - 2, "dual_cold": len(cold) - 2,
                     "mgs_steps": steps, "solves_r0": solves},
        "bytes_per_launch": {
            "dual_solver": statistics.mean(byte[d] for d in solver_dual),
            "dual_warm": statistics.mean(byte[d] for d in warm[2:]),
            "dual_cold": statistics.mean(byte[d] for d in cold[2:]),
            "mgs_solver": mgs_bytes / steps if steps else None,
        },
        "kernel_names": sorted({names[d] for d in solver_dual} | {names[d] for d in mgs}),
    }
    # the constrained step's full reduction (round 5): the basis transpose and the K7t / K7m Gram
    for key, pat in (("transpose", "transpose_basis"), ("gram_sym", "constraint_gram_sym_kernel"),
                     ("gram_mfma", "constraint_gram_mfma_kernel")):
        ds = [d for d in byte if d <= end_solver and pat in names[d]]
        if ds:
            res["bytes_per_launch"][key] = statistics.mean(byte[d] for d in ds)
            res["launches"][key] = len(ds)
    a = argparse.Namespace(config=cfg, spmv_pipe="auto", col16=1, slab_key=1, chain=3, nt_basis=2, orthog="mgs",
                           no_fuse=False, M=None)
    wl = bench.build_workload(argparse.Namespace(config=cfg, M=None, cycles=1))
    nnz = wl["A"].nnz
    c16 = 12 * nnz > 256 * 1024 * 1024 and cfg in ("c3", "c5")
    pipe = "xcd" if cfg in ("c3", "c5") or 12 * nnz <= 256 * 1024 * 1024 else "stride"
    res["options"] = {"spmv_pipe": pipe, "col16": bool(c16), "slab_key": a.slab_key, "chain": a.chain,
                      "nt_basis": a.nt_basis, "orthog": a.orthog, "fuse": True}
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1)
    print(json.dumps(res["bytes_per_launch"]), json.dumps(res["launches"]))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["run", "reduce"])
    ap.add_argument("cfg", choices=["c2", "c3", "c4", "c5"])
    ap.add_argument("files", nargs="*")
    a = ap.parse_args()
    if a.what == "run":
        steps = "1" if a.cfg == "c5" else "3"
        sys.argv = ["bench.py", "--config", a.cfg, "--steps", steps, "--warmup", "1", "--no-cpu-baseline", "--no-wrapper"]
        import bench

        bench.main()
    else:
        reduce(a.cfg, *a.files)
