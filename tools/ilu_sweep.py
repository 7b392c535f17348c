"""Time the device ILU apply (K8) against SuperLU's host solve on the reference's preconditioners
(swe/TimedSolve.py:23 drop 1e-2; lkdvRK/Evolve.py:51 drop 1e-4).  Env SPIS_ILU_GRID /
SPIS_ILU_SLEEP (read once per process) select launch parameters for sweeps; prints one JSON
line per case."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import scipy.sparse.linalg as spsla

from structurepreservingiterativesolvers_amd import device
from structurepreservingiterativesolvers_amd.lkdvRK import assembly as ra
from structurepreservingiterativesolvers_amd.swe import assembly as sa


def cases(which):
    for w in which.split(","):
        kind, m = w.split(":")
        m = int(m)
        if kind == "swe":
            yield f"swe_M{m}", sa.linforms(M=m)[0]["A"], 1e-2
        elif kind == "rk":
            yield f"lkdvRK_M{m}_s3", ra.linforms(M=m, tstages=3)[0]["A"], 1e-4


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "swe:128,swe:256,rk:2000"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    ctx = device.get_context()
    for name, A, drop in cases(which):
        t = time.perf_counter()
        P = spsla.spilu(A.tocsc(), drop_tol=drop, fill_factor=10)
        t_fact = time.perf_counter() - t
        t = time.perf_counter()
        d = device.DeviceILU(ctx, P)
        t_plan = time.perf_counter() - t
        n = A.shape[0]
        qh = np.random.default_rng(0).standard_normal(n)
        q = device.DeviceVector.from_host(qh, ctx=ctx)
        z = device.DeviceVector(ctx, n)
        for _ in range(3):
            d.apply(q, z)
        t = time.perf_counter()
        for _ in range(reps):
            d.apply(q, z)
        t_dev = (time.perf_counter() - t) / reps
        t = time.perf_counter()
        hr = max(1, min(reps, 5))
        for _ in range(hr):
            ref = P.solve(qh)
        t_host = (time.perf_counter() - t) / hr
        err = float(np.linalg.norm(z.numpy() - ref) / np.linalg.norm(ref))
        print(json.dumps({"case": name, "n": n, "device_ms": round(t_dev * 1e3, 4), "host_ms": round(t_host * 1e3, 4),
                          "factor_s": round(t_fact, 3), "plan_s": round(t_plan, 3), "rel_err": err, **d.info}),
              flush=True)


if __name__ == "__main__":
    main()
