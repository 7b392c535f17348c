"""Drop-in for the reference ``lkdvRK/Evolve.py:19-92``: ``N`` Gauss-Legendre steps.  Each
stage solve warm-starts from the previous step's stage vector (``x0 = z``, ``:62``; the first
from ``tile(z0, s)``, ``:36``), the new state is ``z1calc`` (``:70-71``), and the u-error against
the exact travelling wave is recorded (``:80-81``, ``lkdvRK/lkdvRK.py:223-240``).

``pre`` defaults to the reference's host ``spilu(A, drop_tol=1e-4, fill_factor=10)`` (``:48-49``),
built once (the stage operator is the same every step); ``pre=None`` runs unpreconditioned,
and any object ``solvers.cgmres`` accepts as ``pre`` is passed through.  ``degree`` defaults to 3
as in the reference (``:19``); the synthetic assembly is DG(q) with an equispaced Lagrange basis
(``lkdv/assembly.py`` ``dg_operators``), SURVEY §8 config C4 is its q = 1 case."""
import numpy as np
import scipy.sparse.linalg as spsla

from .. import _evolve
from . import LinearSolver as ls
from . import assembly as asm

_SPILU = object()


def compute_error(forms, prob, zbig, t):
    """``lkdvRK/lkdvRK.py:223-240``: L2 norm of ``I(u_exact(t)) - u1`` with the exact solution
    interpolated at the DG(q) nodes (dof (q+1) c + i at ``(c + i/q) h``; q = 1: the cell end
    points)."""
    nf = forms["_step"]["nf"]
    Mass = forms["_step"]["Mass"]
    z1 = asm.z1calc(prob, zbig, forms["z0"])
    q = int(prob.degree)
    M = nf // (q + 1)
    h = prob.mlength / M
    xn = ((np.arange(M)[:, None] + np.arange(q + 1)[None, :] / q) * h).reshape(-1)
    e = prob.exact(xn, t) - z1[:nf]
    return float(np.sqrt(e @ (Mass @ e)))


def evolve(N=10, M=50, degree=3, tstages=2, T=1, k=50, tol=1e-6, contol=10, solver=ls.cgmresWrapper,
           pre=_SPILU):
    forms, prob = asm.linforms(N=N, M=M, degree=degree, tstages=tstages, T=T)
    if pre is _SPILU:
        pre = spsla.spilu(forms["A"].tocsc(), drop_tol=1e-4, fill_factor=10)
    x_init = np.tile(forms["z0"], prob.ns)

    def solve(f, x):
        return solver(f, x0=x_init if x is None else x, prob=prob, pre=pre, k=k, tol=tol, contol=contol)

    return _evolve.run(
        forms, prob, N, asm.step_forms,
        solve=solve,
        state=lambda f, x: asm.z1calc(prob, x, f["z0"]),
        invariants=lambda f, x: asm.compute_invariants(prob, f, x),
        names=[("mass", "m0"), ("momentum", "mo0"), ("energy", "e0")],
        dt_out=forms["T"] / N,
        extra=lambda f, x, t: compute_error(f, prob, x, t),
    )
