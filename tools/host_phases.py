"""GPU: the host time of a C3 solve call as the bench makes it (device matrix, vectors and
constraints resident), split into the Python wrapper's phases (solvers._CHECKPOINTS) and
spis_solve's own (a library built with -DSPIS_HOST_PHASES: `make phases`).

    SPIS_LIBRARY=tools/libspis_phases.so python tools/host_phases.py [solves]
"""
import argparse
import gc
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402
from structurepreservingiterativesolvers_amd import solvers  # noqa: E402
from structurepreservingiterativesolvers_amd.device import (DeviceVector, device_constraints,  # noqa: E402
                                                            device_matrix, get_context)

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 80
cfg = sys.argv[2] if len(sys.argv) > 2 else "c3"
wl = bench.build_workload(argparse.Namespace(config=cfg, M=None, cycles=10))
ctx = get_context(0)
Ad = device_matrix(wl["A"], ctx=ctx)
bd = DeviceVector.from_host(wl["b"], ctx=ctx)
x0d = DeviceVector.from_host(np.zeros(Ad.shape[0]), ctx=ctx)
conlist = device_constraints(wl["conlist"], ctx=ctx)


def solve():
    return solvers.cgmres(Ad, bd, x0d, 30, tol=1e-19, conlist=conlist)  # (C4's lifted constraints: class form)


for _ in range(5):
    _, d = solve()
gc.collect()
gc.freeze()
import ctypes as C  # noqa: E402

t_fn = getattr(ctx.L, "spis_debug_phase_t", None)
if t_fn is not None:
    t_fn.restype = C.c_double
    t_fn.argtypes = [C.c_int]
solvers._CHECKPOINTS = cps = []
marks = []
entry = []
for _ in range(reps):
    t = time.perf_counter()
    _, d = solve()
    marks.append((t, time.perf_counter(), d["x"].stamps[4 * 30], d["x"].stamps[4 * 30 + 1]))
    entry.append([t_fn(i) for i in range(40)] if t_fn is not None else [np.nan] * 40)
solvers._CHECKPOINTS = None
ph = np.array(cps).reshape(reps, 5)
m = np.array(marks)
print("per call %.1f us, between the C stamps %.1f us" % (1e6 * np.mean(m[:, 1] - m[:, 0]),
                                                         1e6 * np.mean(m[:, 3] - m[:, 2])))
print("cgmres entry -> _run entry %.1f us" % (1e6 * np.mean(ph[:, 0] - m[:, 0])))
for i, name in enumerate(["setup (matrix, vectors, constraints, opts)", "buffers + scratch", "spis_solve call",
                          "results + IterateList"]):
    print("%-44s %.1f us" % (name, 1e6 * np.mean(ph[:, i + 1] - ph[:, i])))
print("spis_solve call: entry -> t_start %.1f us, t_end -> return %.1f us" % (
    1e6 * np.mean(m[:, 2] - ph[:, 2]), 1e6 * np.mean(ph[:, 3] - m[:, 3])))
P = np.array(entry)
e = P[:, 0]
print("python -> C entry %.1f us, C entry -> t_start %.1f us" % (1e6 * np.mean(e - ph[:, 2]), 1e6 * np.mean(m[:, 2] - e)))
dP = 1e6 * np.diff(P[:, :10], axis=1)
print("spis_solve marks, per call (us): mean", np.round(dP.mean(axis=0), 1), "max", np.round(dP.max(axis=0), 1))
print("t_start - mark 4 (us): mean %.2f" % (1e6 * np.mean(m[:, 2] - P[:, 4])))
# the last iteration (j = k - 1): H column read (10), KKT block (11 wait start, 12 values in,
# 13 assembled, 14 KKT solved), the GEMV enqueue (15, 16)
L10 = 1e6 * np.diff(P[:, 10:17], axis=1)
print("last iteration, mark 10 -> 16 deltas (us): mean", np.round(L10.mean(axis=0), 1), "median",
      np.round(np.median(L10, axis=0), 1))
# iteration SPIS_PHASE_ITER (10): wait for H[:, j] (20 -> 21), Givens (-> 22), enqueue c_11 (-> 23), LS and
# branch (-> 24), wait for res_9 (-> 25), (-> 26), enqueue the dual (-> 27)
L20 = 1e6 * np.diff(P[:, 20:28], axis=1)
print("iteration %s, mark 20 -> 27 deltas (us): mean" % os.environ.get("SPIS_PHASE_ITER", "10"), np.round(L20.mean(axis=0), 1), "median",
      np.round(np.median(L20, axis=0), 1))
# the start-up launches (marks 4 -> 30 copy_flag, -> 31 r0 SpMV, -> 32 normalize, -> 33 A_0 SpMV + chain,
# -> 34 A_1 SpMV, 34 -> 5 the wait for beta)
S0 = 1e6 * np.diff(P[:, [4, 30, 31, 32, 33, 34, 5]], axis=1)
print("start-up, mark 4 -> 30 -> 31 -> 32 -> 33 -> 34 -> 5 deltas (us): mean", np.round(S0.mean(axis=0), 1))
# the ctypes call alone: spis_solve with a null context returns at its argument check
opts, out, ws = solvers._lib.SolveOpts(), solvers._lib.SolveOut(), C.c_void_p()
t = time.perf_counter()
for _ in range(2000):
    ctx.L.spis_solve(None, None, C.c_void_p(5), C.c_void_p(6), C.byref(opts), C.byref(out), C.byref(ws))
print("null-context spis_solve call %.2f us" % (1e6 * (time.perf_counter() - t) / 2000))
print("_run return -> cgmres return + assignment %.1f us" % (1e6 * np.mean(m[:, 1] - ph[:, 4])), flush=True)
