"""swe/TimedSolve.py:18-70 on the GPU: for each M, spilu(A, drop_tol=1e-2, fill_factor=10), then
a preconditioned GMRES and a timed preconditioned CGMRES (k=20, tol=1e-7) through the drop-in
wrappers, with the preconditioner applied on the device (K8) or by the host callback; prints
one JSON line per (M, mode) with the reference's table columns (runtime, iteration times,
constraint building, conservation gains).  `--oracle-max-M` also times the CPU restatement
(the reference's algorithm) for the smaller M.

usage: python tools/timed_solve.py [--M 16,32,64,128,256] [--modes device,host] [--oracle-max-M 32]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import scipy.sparse.linalg as spsla  # noqa: E402

from structurepreservingiterativesolvers_amd import device  # noqa: E402
from structurepreservingiterativesolvers_amd.swe import LinearSolver as ls  # noqa: E402
from structurepreservingiterativesolvers_amd.swe import assembly as sa  # noqa: E402


def conservation(prob, params, x):
    inv = sa.compute_invariants(prob, params, x)
    return abs(inv["mass"] - params["m0"]), abs(inv["energy"] - params["e0"])


def run(M, mode, k, tol, oracle):
    params, prob = sa.linforms(M=M)
    t = time.perf_counter()
    pre = spsla.spilu(params["A"].tocsc(), drop_tol=1e-2, fill_factor=10)
    t_pre = time.perf_counter() - t
    x0 = np.zeros_like(params["b"])
    out = {"M": M, "n": int(params["A"].shape[0]), "mode": mode, "time_pre": t_pre}
    if mode == "oracle":
        from oracle import cgmres_port as port  # CPU restatement of the reference (baseline only)

        t = time.perf_counter()
        gx, _ = port.gmres(params["A"], params["b"], x0, k, tol=tol, pre=pre)
        out["time_gmres"] = time.perf_counter() - t
        cx, d = port.cgmres(params["A"], params["b"], x0, k, tol=tol, conlist=ls.constraints(params, x0), pre=pre,
                            timing=True)
    else:
        ctx = device.get_context()
        device.set_option("device_ilu", mode == "device")
        if mode == "device":
            t = time.perf_counter()
            di = device.device_ilu(pre, ctx)
            out["time_plan"] = time.perf_counter() - t
            out["plan"] = di.info
        ls.gmresWrapper(params, x0=x0, k=k, tol=tol, pre=pre)  # warm: uploads, workspaces and the
        ls.cgmresWrapper(params, x0=x0, k=k, tol=tol, pre=pre)  # constraint matrices' ELL copies
        t = time.perf_counter()
        gx, _ = ls.gmresWrapper(params, x0=x0, k=k, tol=tol, pre=pre)
        out["time_gmres"] = time.perf_counter() - t
        cx, d = ls.cgmresWrapper(params, x0=x0, k=k, tol=tol, pre=pre, timing=True)
        device.set_option("device_ilu", "auto")
    out.update({key: float(v) for key, v in d["timings"].items()})
    out["unconstrained_steps"] = int(d["steps"] - d["timings"]["constrained_steps"])
    gm, ge = conservation(prob, params, np.asarray(gx))
    cm, ce = conservation(prob, params, np.asarray(cx))
    out["mass_gain"] = max(gm, 1e-16) / max(cm, 1e-16)
    out["energy_gain"] = max(ge, 1e-16) / max(ce, 1e-16)
    out["steps"] = int(d["steps"])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", default="16,32,64,128,256")
    ap.add_argument("--modes", default="device,host")
    ap.add_argument("--oracle-max-M", type=int, default=0)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--tol", type=float, default=1e-7)
    a = ap.parse_args()
    for M in [int(v) for v in a.M.split(",")]:
        modes = a.modes.split(",") + (["oracle"] if M <= a.oracle_max_M else [])
        for mode in modes:
            print(json.dumps(run(M, mode, a.k, a.tol, None)), flush=True)


if __name__ == "__main__":
    main()
