"""Drop-in for the reference ``lkdv/LinearSolver.py`` (same signatures).

Constraints (``lkdv/LinearSolver.py:28-47``): mass (``M = 0, v = omega,
c = -m0``), momentum (``M``, ``c = -mo0``), energy (``L - M``, ``c = -e0``).
"""
import warnings

import numpy as np
import scipy.sparse as sps

from .. import solvers
from .._wrapcache import derived, zeros


class _Constraint:
    def __init__(self, M, v, c):
        self.M, self.v, self.c = M, v, c


def constraints(dic, x0):
    A, M, L = dic["A"], dic["M"], dic["L"]
    zero = zeros(len(x0))  # np.zeros_like(x0), shared read-only
    return [
        _Constraint(derived([A], ["zero"], lambda: sps.csr_matrix(A.shape)), np.transpose(dic["omega"]), -dic["m0"]),
        _Constraint(M, zero, -dic["mo0"]),
        _Constraint(derived([L, M], ["L-M"], lambda: L - M), zero, -dic["e0"]),
    ]


def cgmresWrapper(dic, x0, k, tol=1e-50, contol=10, timing=None):
    conlist = constraints(dic, x0)
    if tol > 1e-20:  # lkdv/LinearSolver.py:50
        return solvers.cgmres(A=dic["A"], b=dic["b"], x0=x0, k=k, tol=tol, contol=contol, conlist=conlist,
                              timing=timing)
    if timing is not None:  # :56-57
        raise NotImplementedError("Timings are not available for prototypical solver")
    return solvers.cgmres_p(A=dic["A"], b=dic["b"], x0=x0, k=k, conlist=conlist)


def gmresWrapper(dic, x0, k, tol=1e-50, contol=None):
    if contol is not None:
        warnings.warn("Contol is ignored as not used in GMRES")
    return solvers.gmres(A=dic["A"], b=dic["b"], x0=x0, k=k, tol=tol)


def exact(dic, x0=None, k=None, tol=None, prob=None, contol=None):
    """Direct solve (``lkdv/LinearSolver.py:76-83``): SciPy ``spsolve`` on the host,
    as in the reference (a comparison baseline, not the Krylov path)."""
    return sps.linalg.spsolve(dic["A"], dic["b"]), -1
