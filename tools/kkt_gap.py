"""GPU: where the host time of C3's forced constrained step goes (stamps of spis_solve): the wait
for the constraint reduction + its assembly, then the KKT solve and the GEMV enqueue.

    python tools/kkt_gap.py [solves]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from structurepreservingiterativesolvers_amd import solvers  # noqa: E402
from structurepreservingiterativesolvers_amd.device import DeviceVector, device_constraints, device_matrix, get_context  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
wl = bench.build_workload(argparse.Namespace(config="c3", M=None, cycles=1))
ctx = get_context(0)
A = device_matrix(wl["A"], ctx=ctx)
n = wl["A"].shape[0]
bd = DeviceVector.from_host(wl["b"], ctx=ctx)
x0d = DeviceVector.from_host(np.zeros(n), ctx=ctx)
cons = device_constraints(wl["conlist"], ctx=ctx)
k = 30
rows = []
for r in range(reps + 3):
    _, d = solvers.cgmres(A, bd, x0d, k, tol=1e-19, conlist=cons)
    st = d["x"].stamps
    j = k - 1
    t_iter0, t_iter1 = st[j], st[k + j]          # iteration j start / end (res read)
    c0, c1 = st[2 * k + j], st[3 * k + j]        # constraint terms: start / end
    call0, call1 = st[4 * k], st[4 * k + 1]
    if r >= 3:
        rows.append((c1 - c0, call1 - c1, call1 - call0, t_iter1 - t_iter0 if t_iter0 > 0 else float("nan")))
a = np.array(rows) * 1e6
print("per solve (us, median over %d): terms wait+assembly %.1f | from terms to the call's end %.1f | call %.1f" %
      (reps, np.median(a[:, 0]), np.median(a[:, 1]), np.median(a[:, 2])))
