"""GPU: where the host time of a C3 solve call goes outside spis_solve (the Python wrapper and
its result objects): cProfile over repeated solves of the bench's C3 workload.

    python tools/host_overhead.py [solves]
"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402
from structurepreservingiterativesolvers_amd import solvers  # noqa: E402
from structurepreservingiterativesolvers_amd.device import DeviceVector, device_constraints, get_context  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
import argparse  # noqa: E402

wl = bench.build_workload(argparse.Namespace(config="c3", M=None, cycles=10))
ctx = get_context(0)
A = wl["A"]
bd = DeviceVector.from_host(wl["b"], ctx=ctx)
x0d = DeviceVector.from_host(np.zeros(A.shape[0]), ctx=ctx)
conlist = device_constraints(wl["conlist"], ctx=ctx)


def solve():
    return solvers.cgmres(A, bd, x0d, 30, tol=1e-19, conlist=conlist)


orig = ctx.L.spis_solve
acc = {"c": 0.0}


def timed(*a):
    t = time.perf_counter()
    r = orig(*a)
    acc["c"] += time.perf_counter() - t
    return r


ctx.L.spis_solve = timed
orig_rel = ctx.L.spis_workspace_release
acc["r"] = 0.0


def timed_rel(*a):
    t = time.perf_counter()
    r = orig_rel(*a)
    acc["r"] += time.perf_counter() - t
    return r


ctx.L.spis_workspace_release = timed_rel
for _ in range(3):
    solve()
out = inner = 0.0
acc["c"] = acc["r"] = 0.0
for _ in range(reps):
    t = time.perf_counter()
    _, d = solve()
    st = d["x"].stamps
    out += time.perf_counter() - t
    inner += st[4 * 30 + 1] - st[4 * 30]
print(f"per call: total {1e6 * out / reps:.1f} us, spis_solve {1e6 * acc['c'] / reps:.1f} us, "
      f"stamped solve {1e6 * inner / reps:.1f} us -> Python {1e6 * (out - acc['c']) / reps:.1f} us, "
      f"C outside the stamps {1e6 * (acc['c'] - inner) / reps:.1f} us; workspace release "
      f"{1e6 * acc['r'] / reps:.1f} us", flush=True)
pr = cProfile.Profile()
pr.enable()
for _ in range(reps):
    _, d = solve()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)

# the wrapper's pieces, one at a time
from structurepreservingiterativesolvers_amd import _lib  # noqa: E402
from structurepreservingiterativesolvers_amd.device import device_matrix, device_vector  # noqa: E402


def tm(name, f, n=200):
    f()
    t = time.perf_counter()
    for _ in range(n):
        f()
    print(f"{name:32s} {1e6 * (time.perf_counter() - t) / n:8.1f} us", flush=True)


n = A.shape[0]
tm("device_matrix(A)", lambda: device_matrix(A, ctx=ctx))
tm("device_vector(bd)", lambda: device_vector(bd, ctx=ctx))
tm("_constraint_desc x2", lambda: [solvers._constraint_desc(c, n, ctx) for c in conlist])
tm("_precond_setup", lambda: solvers._precond_setup(None, n, ctx, []))
tm("kinds check", lambda: ["class" if hasattr(c, "__dict__") else "dict" if type(c) is dict else "bad" for c in conlist])
tm("scratch + drop", lambda: DeviceVector.scratch(ctx, n))
tm("_out_buffers + fill", lambda: [b.fill(0) for b in solvers._out_buffers(30)[:2]])
_, d0 = solve()
xs0 = d0["x"]
tm("d['x'] trace", lambda: xs0.events.any())
tm("IterateList(no ws)", lambda: solvers.IterateList(ctx, None, n, 31, None))
print("events of a C3 solve:", xs0.events, flush=True)
import warnings  # noqa: E402

tm("warnings.warn (repeat)", lambda: warnings.warn("Iteration 29 failed with message 'x'", RuntimeWarning))

# _run's phases: [entry, before the output buffers, before spis_solve, after it, before return]
solvers._CHECKPOINTS = cps = []
marks = []
for _ in range(reps):
    t = time.perf_counter()
    _, d = solve()
    marks.append((t, time.perf_counter()))
solvers._CHECKPOINTS = None
ph = np.array(cps).reshape(reps, 5)
m = np.array(marks)
print("cgmres entry -> _run entry %.1f us" % (1e6 * np.mean(ph[:, 0] - m[:, 0])))
for i, name in enumerate(["setup (matrix, vectors, constraints, opts)", "buffers + scratch", "spis_solve",
                          "results + IterateList"]):
    print("%-44s %.1f us" % (name, 1e6 * np.mean(ph[:, i + 1] - ph[:, i])))
print("_run return -> cgmres return + assignment %.1f us" % (1e6 * np.mean(m[:, 1] - ph[:, 4])), flush=True)
