"""Drop-in for the reference ``swe/LinearSolver.py`` (same signatures).

Constraints (``swe/LinearSolver.py:23-36``): mass (``M = 0, v = omega,
c = -m0``) and energy (``M = L, c = -e0``).
"""
import numpy as np
import scipy.sparse as sps

from .. import solvers
from .._wrapcache import derived, zeros


class _Constraint:
    def __init__(self, M, v, c):
        self.M, self.v, self.c = M, v, c


def constraints(dic, x0):
    A = dic["A"]
    return [
        _Constraint(derived([A], ["zero"], lambda: sps.csr_matrix(A.shape)), np.transpose(dic["omega"]), -dic["m0"]),
        _Constraint(dic["L"], zeros(len(x0)), -dic["e0"]),  # np.zeros_like(x0), shared read-only
    ]


def cgmresWrapper(dic, x0, k, tol=1e-50, pre=None, timing=None):
    conlist = constraints(dic, x0)
    if tol < 1e-20:  # swe/LinearSolver.py:40
        return solvers.cgmres_p(A=dic["A"], b=dic["b"], x0=x0, k=k, conlist=conlist, pre=pre)
    return solvers.cgmres(A=dic["A"], b=dic["b"], x0=x0, k=k, tol=tol, conlist=conlist, timing=timing, pre=pre)


def gmresWrapper(dic, x0, k, tol=1e-50, pre=None):
    return solvers.gmres(A=dic["A"], b=dic["b"], x0=x0, k=k, tol=tol, pre=pre)
