"""Constraint terms of the swe test case (M=30, k=25) on an MGS Arnoldi basis, from each K7 form,
against an exactly rounded host reference (math.fsum of exact products): which form's terms are
closer, entry by entry.  python tools/diag_terms.py"""
import math
import sys
from fractions import Fraction

import numpy as np

sys.path.insert(0, ".")
from structurepreservingiterativesolvers_amd import solvers  # noqa: E402
from structurepreservingiterativesolvers_amd.device import set_option  # noqa: E402
from structurepreservingiterativesolvers_amd.swe import LinearSolver as swe_ls  # noqa: E402
from structurepreservingiterativesolvers_amd.swe import assembly as sa  # noqa: E402

dic, _ = sa.linforms(M=30)
A, b = dic["A"], dic["b"]
k = 25
n = len(b)
Q = np.zeros((k + 1, n))
Q[0] = b / np.linalg.norm(b)
for j in range(k):
    y = A @ Q[j]
    for i in range(j + 1):
        y = y - (Q[i] @ y) * Q[i]
    Q[j + 1] = y / np.linalg.norm(y)
Z = Q[:k].T.copy()
x0 = np.zeros(n)
cons = swe_ls.constraints(dic, x0)


def exact_dot(u, v):
    return float(sum(Fraction(a) * Fraction(c) for a, c in zip(u, v)))


L = dic["L"]
LZ = [None] * k
res = {}
for mode in ("ell", "mfma", "mfma_full"):
    set_option("ell_gram", mode)
    res[mode] = [solvers.constraint_container(c, x0, Z) for c in cons]
set_option("ell_gram", "mfma")
# exact term1 of the mass constraint (v = omega) and a few term2 entries of the energy one
om = dic["omega"]
t1 = np.array([math.fsum(om * Z[:, a]) for a in range(k)])
for mode, cc in res.items():
    print(mode, "mass term1 max |err| / max|t1|", np.abs(cc[0].term1 - t1).max() / np.abs(t1).max(),
          "err on a>=1 rel to sum|om z|", np.abs(cc[0].term1[1:] - t1[1:]).max() / np.abs(om) @ np.abs(Z[:, 1]))
LZ = (L @ Z)
for a in (0, 1, 5, 24):
    for bb in (0, 3, 24):
        ex = 0.5 * math.fsum(Z[:, a] * LZ[:, bb])
        print(a, bb, "exact-ish", ex, {m: (cc[1].term2[a, bb] - ex) / abs(ex) for m, cc in res.items()})
print("term1 energy", {m: np.abs(cc[1].term1).max() for m, cc in res.items()})
print("term0", {m: (cc[0].term0, cc[1].term0) for m, cc in res.items()})
print("mass term1", {m: cc[0].term1[:4] for m, cc in res.items()}, t1[:4])
