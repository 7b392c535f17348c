"""GPU: K7t (symmetric constraint Gram from the slot table) at 16 and 32 slots against K7m on
the same inputs, over matrices of growing size (blocks per wave from < 1 to many) and simple
structures (diagonal, tridiagonal, the swe energy matrix), to localise a slot-count-dependent
error:

    python tools/k7t_probe.py

One line per case: n, table blocks at 16 / 32 slots (estimated on the host), max relative
error of term2 for each slot count."""
import os
import sys

import numpy as np
import scipy.sparse as sps

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from structurepreservingiterativesolvers_amd import solvers  # noqa: E402
from structurepreservingiterativesolvers_amd.device import set_option  # noqa: E402
from structurepreservingiterativesolvers_amd.swe import assembly as sa  # noqa: E402


class Con:
    pass


def gram(Mv, Z, x0, mode, slots):
    con = Con()
    con.M, con.v, con.c = Mv, np.zeros(Mv.shape[0]), 0.0
    set_option("ell_gram", mode)
    set_option("k7t_slots", slots)
    try:
        return solvers.constraint_container(con, x0, Z).term2
    finally:
        set_option("ell_gram", "mfma")
        set_option("k7t_slots", 16)


def case(name, Mv, p=31, seed=3):
    Mv = sps.csr_matrix(Mv)
    n = Mv.shape[0]
    rng = np.random.default_rng(seed)
    Z = rng.normal(size=(n, p))
    x0 = rng.normal(size=n)
    ref = gram(Mv, Z, x0, "mfma_full", 16)
    out = [f"{name:28s} n={n:9d}"]
    for slots in (16, 32):
        g = gram(Mv, Z, x0, "mfma", slots)
        err = np.abs(g - ref).max() / np.abs(ref).max()
        out.append(f"slots={slots}: {err:.2e}")
    print("  ".join(out), flush=True)


for n in (64, 1024, 20000, 200000):
    case("diagonal", sps.diags(np.arange(1, n + 1, dtype=float)))
    case("tridiagonal", sps.diags([np.full(n - 1, -1.0), np.full(n, 2.0), np.full(n - 1, -1.0)], [-1, 0, 1]))
for k in (20, 60):
    e = np.ones(4000)
    case(f"band half-width {k}", sps.diags([e[: 4000 - abs(d)] * (1.0 + 0.01 * abs(d)) for d in range(-k, k + 1)],
                                          list(range(-k, k + 1))))
for M in (4, 8, 16, 32, 64, 128):
    dic, _ = sa.linforms(M=M)
    case(f"swe L M={M}", dic["L"])

# timing at C3 (run under rocprofv3 --kernel-trace --stats: constraint_gram_sym_kernel<16> / <32>)
if len(sys.argv) > 1 and sys.argv[1] == "time":
    dic, _ = sa.linforms(M=289)
    Mv = sps.csr_matrix(dic["L"])
    rng = np.random.default_rng(5)
    Z = rng.normal(size=(Mv.shape[0], 31))
    x0 = rng.normal(size=Mv.shape[0])
    for slots in (16, 32):
        for _ in range(10):
            gram(Mv, Z, x0, "mfma", slots)
        print(f"C3 timed at {slots} slots", flush=True)
