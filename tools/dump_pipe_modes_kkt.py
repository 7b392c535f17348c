"""GPU: the swe M=30 CGMRES(25) solve of tests/test_gpu_parity.py::test_spmv_pipe_modes_solver_agree
under every SpMV kernel family, dumping each run's constrained-step inputs (H, beta, warm start,
reduced terms) and outcome for host-side KKT analysis:  python tools/dump_pipe_modes_kkt.py OUTDIR"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from structurepreservingiterativesolvers_amd import solvers  # noqa: E402
from structurepreservingiterativesolvers_amd.device import set_option  # noqa: E402
from structurepreservingiterativesolvers_amd.swe import LinearSolver as swe_ls  # noqa: E402
from structurepreservingiterativesolvers_amd.swe import assembly as sa  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pipekkt"
os.makedirs(out, exist_ok=True)
dic, _ = sa.linforms(M=30)
cons = swe_ls.constraints(dic, np.zeros_like(dic["b"]))
k = 25
for pipe in ("off", "stride", "xcd", "xcd_natural"):
    set_option("spmv_pipe", pipe)
    x, d = solvers.cgmres(dic["A"], dic["b"], np.zeros_like(dic["b"]), k, tol=1e-19, conlist=cons)
    xs = d["x"]
    terms = [xs.constraint_terms(i) for i in range(len(cons))]
    np.savez(os.path.join(out, f"kkt_{pipe}.npz"), H=xs.hessenberg(k), beta=xs.beta,
             y0=np.concatenate([xs.y[k - 2], [0.0]]), y_dev=xs.y[k - 1], branch=xs.trace[-1][1],
             t0=np.array([t[1] for t in terms]), t1=np.stack([t[2] for t in terms]), t2=np.stack([t[3] for t in terms]))
    print(pipe, xs.trace[-1], int(xs.events[-1]), d["res"][-1], flush=True)
set_option("spmv_pipe", "auto")
