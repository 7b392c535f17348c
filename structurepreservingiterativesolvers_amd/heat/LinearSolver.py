"""Drop-in for the reference ``heat/LinearSolver.py`` (same signatures).

Constraints (``heat/LinearSolver.py:26-38``): mass ``M = 0, v = omega,
c = -m0`` and the dissipation-matched energy ``M = Mass + dt/2 L,
v = dt/2 Lz0, c = -old_energy``.  The zero mass matrix is an empty CSR (the
reference's ``0*A`` stores A's whole pattern as explicit zeros and pays a full
SpMM of zeros, SURVEY finding 8); the values are identical.
"""
import numpy as np
import scipy.sparse as sps

from .. import solvers
from .._wrapcache import derived


class _Constraint:
    def __init__(self, M, v, c):
        self.M, self.v, self.c = M, v, c


def constraints(dic):
    A, dt, M, L = dic["A"], dic["dt"], dic["M"], dic["L"]
    mass = _Constraint(derived([A], ["zero"], lambda: sps.csr_matrix(A.shape)), np.transpose(dic["omega"]), -dic["m0"])
    energy = _Constraint(derived([M, L], ["heat_energy", dt], lambda: M + 0.5 * dt * L), 0.5 * dt * dic["Lz0"],
                         -dic["old_energy"])
    return [mass, energy]


def cgmresWrapper(dic, x0, k, tol=1e-50, pre=None, timing=None):
    conlist = constraints(dic)
    if tol < 1e-20:  # heat/LinearSolver.py:43
        return solvers.cgmres_p(A=dic["A"], b=dic["b"], x0=x0, k=k, conlist=conlist, pre=pre)
    return solvers.cgmres(A=dic["A"], b=dic["b"], x0=x0, k=k, tol=tol, conlist=conlist, pre=pre, timing=timing)


def gmresWrapper(dic, x0, k, tol=1e-50, pre=None):
    return solvers.gmres(A=dic["A"], b=dic["b"], x0=x0, k=k, tol=tol, pre=pre)
