"""A/B of the drop-in call (C3 cgmresWrapper, bench.py's wrapper_rate) with x0's all-zero verdict
scanned inline on every call ("inline", rounds 1-6) or cached and re-checked beside the solve
("cached", device.host_x0_zero), alternated on one box."""
import argparse
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
from structurepreservingiterativesolvers_amd import device, solvers  # noqa: E402
from structurepreservingiterativesolvers_amd.swe import LinearSolver as ls  # noqa: E402

args = argparse.Namespace(config="c3", M=None, cycles=1, k=30, tol=1e-19)
dic = bench.build_workload(args)["dic"]
x0 = np.zeros(dic["A"].shape[0])
cached = solvers.host_x0_zero


def inline(a, checks=None):
    return not device.host_nonzero(a, bitwise=True)


for _ in range(3):
    ls.cgmresWrapper(dic, x0, 30, tol=1e-19)
for rnd in range(4):
    for mode, fn in (("inline", inline), ("cached", cached)):
        solvers.host_x0_zero = fn
        solvers._PHASES = {}
        its = 0
        t0 = time.perf_counter()
        for _ in range(30):
            its += ls.cgmresWrapper(dic, x0, 30, tol=1e-19)[1]["steps"]
        el = time.perf_counter() - t0
        ph, solvers._PHASES = solvers._PHASES, None
        print(f"round {rnd} {mode:6s} it/s={its / el:8.1f} ms/call={1e3 * el / 30:.3f} "
              f"h2d={1e3 * ph['h2d'] / 30:.3f} verify_wait={1e3 * ph['verify_wait'] / 30:.3f}", flush=True)
