"""GPU diagnostic (round 4): config C2 (lkdv M=16,667) against the oracle, per iterate, for every MGS
chain mode, beside the reference's own 8-seed roundoff envelope (b perturbed by 1e-16) and the
oracle's sensitivity to the summation order of its MGS dots (the same oracle with every dot
product accumulated in reverse element order).

    python tools/r04_c2_diag.py [M]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import oracle
    from structurepreservingiterativesolvers_amd import solvers
    from structurepreservingiterativesolvers_amd.device import set_option
    from structurepreservingiterativesolvers_amd.lkdv import LinearSolver as ls
    from structurepreservingiterativesolvers_amd.lkdv import assembly as la

    M = int(sys.argv[1]) if len(sys.argv) > 1 else 16667
    dic, _ = la.linforms(M=M)
    A, b = dic["A"], dic["b"]
    x0 = np.zeros_like(b)
    k = 30
    cons = ls.constraints(dic, x0)
    _, d0 = oracle.cgmres(A, b, x0, k, tol=1e-19, conlist=cons)
    ref = np.asarray(d0["x"])
    nr = np.linalg.norm(ref, axis=1)
    env = np.zeros(len(ref))
    for sd in range(8):
        bp = b * (1 + 1e-16 * np.random.default_rng(sd).normal(size=b.shape))
        _, dp = oracle.cgmres(A, bp, x0, k, tol=1e-19, conlist=cons)
        xp = np.asarray(dp["x"])
        env = np.maximum(env, np.linalg.norm(xp - ref, axis=1) / nr)
    rows = {"env8": env}
    for mode in ("pipelined", "aggregator", "one_reduce", False):
        set_option("mgs_chain", mode)
        _, d = solvers.cgmres(A, b, x0, k, tol=1e-19, conlist=cons)
        xs = np.asarray(d["x"])
        rows[str(mode)] = np.linalg.norm(xs - ref, axis=1) / nr
    set_option("mgs_chain", "pipelined")
    print("i " + " ".join(f"{n:>11s}" for n in rows))
    for i in range(len(ref)):
        print(f"{i:2d} " + " ".join(f"{rows[n][i]:11.2e}" for n in rows))


if __name__ == "__main__":
    main()
