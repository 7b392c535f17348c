"""Constraint terms (solvers.py:33-36) of the swe energy matrix at a given mesh size from every K7
form, compared with the sliced-ELL kernel and timed: python tools/gram_check.py [M] [p]"""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from structurepreservingiterativesolvers_amd import solvers  # noqa: E402
from structurepreservingiterativesolvers_amd.device import set_option  # noqa: E402
from structurepreservingiterativesolvers_amd.swe import assembly  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 289
p = int(sys.argv[2]) if len(sys.argv) > 2 else 30
dic, _ = assembly.linforms(M=M)
n = dic["A"].shape[0]
rng = np.random.default_rng(3)
Z = rng.normal(size=(n, p)) / np.sqrt(n)
x0 = rng.normal(size=n)


class Con:
    pass


con = Con()
con.M, con.v, con.c = dic["L"], dic["omega"], -dic["e0"]
res = {}
for mode in ("ell", "mfma_full", "mfma"):
    set_option("ell_gram", mode)
    solvers.constraint_container(con, x0, Z)  # one-time tables
    t0 = time.perf_counter()
    cc = solvers.constraint_container(con, x0, Z)
    dt = time.perf_counter() - t0
    res[mode] = cc
    print(f"{mode:12s} {dt * 1e6:9.1f} us (host wall incl. transfers)")
set_option("ell_gram", "mfma")
ref = res["ell"]
for mode, cc in res.items():
    e2 = np.abs(cc.term2 - ref.term2).max() / np.abs(ref.term2).max()
    e1 = np.abs(cc.term1 - ref.term1).max() / max(np.abs(ref.term1).max(), 1e-300)
    e0 = abs(cc.term0 - ref.term0) / max(abs(ref.term0), 1e-300)
    print(f"{mode:12s} rel err term2 {e2:.2e} term1 {e1:.2e} term0 {e0:.2e}")
