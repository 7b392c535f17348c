"""cProfile of the host side of repeated bench solves (where the Python time outside spis_solve
goes).  usage: python tools/host_profile.py [c2|c3|c4]"""
import argparse
import cProfile
import os
import pstats
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from structurepreservingiterativesolvers_amd import solvers  # noqa: E402
from structurepreservingiterativesolvers_amd.device import (DeviceVector, device_constraints,  # noqa: E402
                                                            device_matrix, get_context)

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
args = argparse.Namespace(config=cfg, M=None, cycles=1)
wl = bench.build_workload(args)
A = wl["A"]
ctx = get_context(0)
device_matrix(A, ctx=ctx)
bd = DeviceVector.from_host(wl["b"], ctx=ctx)
x0d = DeviceVector.from_host(np.zeros(A.shape[0]), ctx=ctx)
cons = device_constraints(wl["conlist"], ctx=ctx)
for _ in range(3):
    solvers.cgmres(A, bd, x0d, 30, tol=1e-19, conlist=cons)
pr = cProfile.Profile()
pr.enable()
for _ in range(20):
    x, d = solvers.cgmres(A, bd, x0d, 30, tol=1e-19, conlist=cons)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
