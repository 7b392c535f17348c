"""C5 probe (round 4): one assembly of the C5 workload, then restarted CGMRES(30) x cycles timed
under several MGS configurations in the same process (options by name, spis_set_option).

  python tools/r04_c5_probe.py --configs "mgs_chain=3,nt_basis=2" "mgs_chain=2,nt_basis=0" ...

Prints one JSON line per configuration: it/s, mean sampled MGS and dual-SpMV launch times.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=913)
    ap.add_argument("--cycles", type=int, default=10)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--configs", nargs="+", default=["mgs_chain=3"])
    args = ap.parse_args()

    from structurepreservingiterativesolvers_amd import _lib, solvers
    from structurepreservingiterativesolvers_amd.device import (DeviceVector, device_constraints, device_matrix,
                                                                get_context, set_option)
    from structurepreservingiterativesolvers_amd.swe import LinearSolver as ls
    from structurepreservingiterativesolvers_amd.swe import assembly

    t0 = time.time()
    dic, _ = assembly.linforms(M=args.M)
    n = dic["A"].shape[0]
    x0 = np.zeros(n)
    cons = ls.constraints(dic, x0)
    D, c3 = assembly.extra_constraint(n, dic["z0"], seed=2)
    cons.append(ls._Constraint(D, np.zeros(n), c3))
    print(json.dumps({"assembly_s": time.time() - t0, "n": n}), flush=True)
    ctx = get_context(0)
    Ad = device_matrix(dic["A"], ctx=ctx)
    bd = DeviceVector.from_host(dic["b"], ctx=ctx)
    x0d = DeviceVector.from_host(x0, ctx=ctx)
    cd = device_constraints(cons, ctx=ctx)
    for cfg in args.configs:
        opts = {}
        for kv in cfg.split(","):
            k, v = kv.split("=")
            opts[k] = v
        for k, v in opts.items():
            val = {"True": True, "False": False}.get(v, v)
            set_option(k, val, ctx)

        def solve():
            return solvers.cgmres_restarted(Ad, bd, x0d, 30, args.cycles, tol=1e-19, conlist=cd)

        x, d = solve()
        ctx.synchronize()
        _lib.check(ctx.L.spis_profile_enable(ctx.handle, 10), "prof")
        t = time.perf_counter()
        iters = 0
        for _ in range(args.steps):
            x, d = solve()
            iters += d["steps"]
        ctx.synchronize()
        dt = time.perf_counter() - t
        ms, cnt = _lib.profile_read(ctx.L, ctx.handle)
        _lib.check(ctx.L.spis_profile_enable(ctx.handle, 0), "prof")
        xh = np.asarray(x)
        branches = [r["x"].trace[-1][1] for r in d["runs"]]
        res = float(np.linalg.norm(dic["A"] @ xh - dic["b"]))
        print(json.dumps({
            "config": cfg, "it_s": iters / dt, "ms_per_solve": 1e3 * dt / args.steps,
            "mgs_us": 1e3 * ms[_lib.PROF_MGS] / max(cnt[_lib.PROF_MGS], 1),
            "dual_us": 1e3 * ms[_lib.PROF_SPMV_DUAL] / max(cnt[_lib.PROF_SPMV_DUAL], 1),
            "gemv_us": 1e3 * ms[_lib.PROF_GEMV] / max(cnt[_lib.PROF_GEMV], 1),
            "final_res": res, "last_branches": branches,
        }), flush=True)
        set_option("mgs_chain", "pipelined", ctx)  # defaults back
        set_option("nt_basis", "auto", ctx)


if __name__ == "__main__":
    main()
