"""Host time per bench solve outside the C solver, split: Python before spis_solve, spis_solve
itself, Python after it, and the time until the next call starts (result drop / finalizers)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from structurepreservingiterativesolvers_amd import solvers  # noqa: E402
from structurepreservingiterativesolvers_amd.device import DeviceVector, device_constraints, device_matrix, get_context  # noqa: E402
from structurepreservingiterativesolvers_amd.swe import LinearSolver as swe_ls  # noqa: E402
from structurepreservingiterativesolvers_amd.swe import assembly  # noqa: E402

dic, _ = assembly.linforms(M=289)
A = dic["A"]
ctx = get_context(0)
device_matrix(A, ctx=ctx)
bd = DeviceVector.from_host(dic["b"], ctx=ctx)
x0d = DeviceVector.from_host(np.zeros(A.shape[0]), ctx=ctx)
cons = device_constraints(swe_ls.constraints(dic, np.zeros(A.shape[0])), ctx=ctx)
real = ctx.L.spis_solve
T = {"in": []}


def timed(*a):
    t = time.perf_counter()
    r = real(*a)
    T["in"].append(time.perf_counter() - t)
    return r


ctx.L.spis_solve = timed
for _ in range(3):
    solvers.cgmres(A, bd, x0d, 30, tol=1e-19, conlist=cons)
T["in"].clear()
walls, keep = [], []
for mode in ("drop", "keep"):
    T["in"].clear()
    walls = []
    for _ in range(20):
        t = time.perf_counter()
        x, d = solvers.cgmres(A, bd, x0d, 30, tol=1e-19, conlist=cons)
        if mode == "keep":
            keep.append(d)
        walls.append(time.perf_counter() - t)
    w = np.array(walls[2:]) * 1e6
    i = np.array(T["in"][2:]) * 1e6
    print(f"{mode}: wall {w.mean():.0f} us, in spis_solve {i.mean():.0f} us, Python around it {(w - i).mean():.0f} us")
    keep.clear()
