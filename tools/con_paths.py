"""Time the constrained step's two device paths (fused K7 vs SpMM + tiled Gram) on the bench
workload: run under rocprofv3 --kernel-trace and compare the kernels of each phase."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from structurepreservingiterativesolvers_amd import _lib, solvers  # noqa: E402
from structurepreservingiterativesolvers_amd.device import (DeviceVector, device_constraints,  # noqa: E402
                                                            device_matrix, get_context)
from structurepreservingiterativesolvers_amd.swe import LinearSolver as swe_ls  # noqa: E402
from structurepreservingiterativesolvers_amd.swe import assembly  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 289
dic, _ = assembly.linforms(M=M)
A = dic["A"]
ctx = get_context(0)
device_matrix(A, ctx=ctx)
bd = DeviceVector.from_host(dic["b"], ctx=ctx)
x0 = np.zeros(A.shape[0])
x0d = DeviceVector.from_host(x0, ctx=ctx)
cons = device_constraints(swe_ls.constraints(dic, x0), ctx=ctx)
out = {}
for mode, flag in (("fused", 0), ("generic", -1), ("fused2", 0)):
    _lib.check(ctx.L.spis_profile_enable(ctx.handle, flag), "spis_profile_enable")
    for _ in range(3):
        x, d = solvers.cgmres(A, bd, x0d, 30, tol=1e-19, conlist=cons)
    out[mode] = (d["res"][-1], np.asarray(d["x"][-1])[:4])
    print(mode, d["res"][-1], flush=True)
print("res fused vs generic", out["fused"][0], out["generic"][0])
