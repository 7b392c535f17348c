"""GPU: run bench.py's C5 workload (swe M, mass + energy + the synthetic third constraint,
restarted CGMRES(k)) cycle by cycle through the device solver, and dump every cycle's
constrained-step inputs as the host KKT received them (H, beta, warm start y0, the three
reduced constraint terms) plus the device's branch, message and y:

    python tools/dump_c5_kkt.py [M] [cycles] [outdir]

The dumps feed tools/c5_branch_probe.py-style checks on the CPU (the reference's SLSQP on the
device's own inputs) and tests/kkt_cases/."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from structurepreservingiterativesolvers_amd import solvers  # noqa: E402
from structurepreservingiterativesolvers_amd.device import DeviceVector, device_constraints, get_context  # noqa: E402
from structurepreservingiterativesolvers_amd.swe import LinearSolver as ls  # noqa: E402
from structurepreservingiterativesolvers_amd.swe import assembly  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 913
cycles = int(sys.argv[2]) if len(sys.argv) > 2 else 10
out = sys.argv[3] if len(sys.argv) > 3 else "gpurun_out/c5kkt"
os.makedirs(out, exist_ok=True)
k = 30
t = time.time()
dic, _ = assembly.linforms(M=M)
n = dic["A"].shape[0]
x0 = np.zeros(n)
cons = ls.constraints(dic, x0)
D, c3 = assembly.extra_constraint(n, dic["z0"], seed=2)
cons.append(ls._Constraint(D, np.zeros(n), c3))
print(f"assembled M={M} N={n} in {time.time() - t:.1f}s", flush=True)
ctx = get_context(0)
bd = DeviceVector.from_host(dic["b"], ctx=ctx)
x = DeviceVector.from_host(x0, ctx=ctx)
cd = device_constraints(cons, ctx=ctx)
for c in range(cycles):
    xn, d = solvers.cgmres(dic["A"], bd, x, k, tol=1e-19, conlist=cd)
    xs = d["x"]
    j = d["steps"] - 1
    tr = xs.trace
    H = xs.hessenberg(j + 1)
    ys = xs.y
    y0 = np.concatenate([ys[j - 1], [0.0]]) if j else np.zeros(1)
    terms = [xs.constraint_terms(i) for i in range(len(cons))]
    path = os.path.join(out, f"kkt_c5_M{M}_cycle{c}.npz")
    np.savez(path, H=H, beta=xs.beta, y0=y0, y_dev=ys[j], branch=tr[-1][1], events=xs.events,
             t0=np.array([tt[1] for tt in terms]), t1=np.stack([tt[2] for tt in terms]),
             t2=np.stack([tt[3] for tt in terms]), res=np.array(d["res"]))
    print(f"cycle {c}: steps={d['steps']} last={tr[-1]} events_last={int(xs.events[-1])} "
          f"res_last={d['res'][-1]:.4e} -> {path}", flush=True)
    xs.release()
    x = xn
