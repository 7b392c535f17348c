"""cProfile of the host side of repeated bench solves (where the Python time outside spis_solve goes)."""
import cProfile
import os
import pstats
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from structurepreservingiterativesolvers_amd import solvers  # noqa: E402
from structurepreservingiterativesolvers_amd.device import (DeviceVector, device_constraints,  # noqa: E402
                                                            device_matrix, get_context)
from structurepreservingiterativesolvers_amd.swe import LinearSolver as swe_ls  # noqa: E402
from structurepreservingiterativesolvers_amd.swe import assembly  # noqa: E402

dic, _ = assembly.linforms(M=int(sys.argv[1]) if len(sys.argv) > 1 else 289)
A = dic["A"]
ctx = get_context(0)
device_matrix(A, ctx=ctx)
bd = DeviceVector.from_host(dic["b"], ctx=ctx)
x0d = DeviceVector.from_host(np.zeros(A.shape[0]), ctx=ctx)
cons = device_constraints(swe_ls.constraints(dic, np.zeros(A.shape[0])), ctx=ctx)
for _ in range(3):
    solvers.cgmres(A, bd, x0d, 30, tol=1e-19, conlist=cons)
pr = cProfile.Profile()
pr.enable()
for _ in range(20):
    x, d = solvers.cgmres(A, bd, x0d, 30, tol=1e-19, conlist=cons)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
