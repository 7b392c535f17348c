"""Drop-in for the reference ``lkdvRK/LinearSolver.py`` (same signatures).

The reference passes its three invariants as dict-form constraints evaluated
on ``X1 = z1calc(x0 + Q y)`` (``lkdvRK/LinearSolver.py:29-79``), so every SLSQP
function evaluation costs an N-length GEMV plus SpMVs.  ``z1calc`` is linear,
``X1 = z0 + P X`` with ``P = dt [b_1 I, ..., b_s I]`` (``lkdvRK/lkdvRK.py:162-174``),
so the same constraints are exactly quadratic in ``X`` and are lifted here to
the class form the device reduces:

* mass:     ``M = 0``,           ``v = P' omega``,          ``c = omega.z0 - m0``
* momentum: ``M = P' M P``,      ``v = P' (M + M')/2 z0``,  ``c = 1/2 z0'M z0 - mo0``
* energy:   ``M = P' K P``,      ``v = P' (K + K')/2 z0``,  ``c = 1/2 z0'K z0 - e0``, ``K = L - M``

``lift=False`` passes the reference's dict-form constraints unchanged (host
SLSQP through the constrained-LS callback of ``spis_solve``).
"""
import warnings

import numpy as np
import scipy.sparse as sps

from .. import solvers
from .._wrapcache import derived
from .assembly import dz1calc, z1calc


class _Constraint:
    def __init__(self, M, v, c):
        self.M, self.v, self.c = M, v, c


def _lift(dic, prob):
    dt = prob.dt
    bw = np.asarray(prob.butcher_tableau.b, dtype=np.float64)
    z0 = np.asarray(dic["z0"], dtype=np.float64)
    M, L, omega = dic["M"], dic["L"], np.asarray(dic["omega"], dtype=np.float64)
    K = derived([L, M], ["L-M"], lambda: L - M)
    PtP = np.outer(dt * bw, dt * bw)

    def Pt(w):
        return np.kron(dt * bw, w)

    n = len(bw) * len(z0)
    # the lifted matrices depend on the operators and the tableau only: built once per problem
    # (time steps share them, so they stay resident in HBM with their sliced-ELL copies)
    key = ["lift", float(dt)] + [float(v) for v in bw]
    zero = derived([M], key + ["zero"], lambda: sps.csr_matrix((n, n)))
    MM = derived([M], key + ["M"], lambda: sps.csr_matrix(sps.kron(PtP, M)))
    KK = derived([L, M], key + ["K"], lambda: sps.csr_matrix(sps.kron(PtP, K)))
    mass = _Constraint(zero, Pt(omega), float(omega @ z0 - dic["m0"]))
    mom = _Constraint(MM, Pt(0.5 * (M @ z0 + M.T @ z0)), float(0.5 * z0 @ (M @ z0) - dic["mo0"]))
    en = _Constraint(KK, Pt(0.5 * (K @ z0 + K.T @ z0)), float(0.5 * z0 @ (K @ z0) - dic["e0"]))
    return [mass, mom, en]


def dict_constraints(dic, prob):
    """The reference's dict-form constraints (``lkdvRK/LinearSolver.py:29-79``)."""
    M, L, omega, z0 = dic["M"], dic["L"], dic["omega"], dic["z0"]
    m0, mo0, e0 = dic["m0"], dic["mo0"], dic["e0"]

    def const1(z, x0, Q):
        return np.transpose(omega) @ z1calc(prob, x0 + Q @ z, z0) - m0

    def const2(z, x0, Q):
        X = z1calc(prob, x0 + Q @ z, z0)
        return 0.5 * np.transpose(X) @ M @ X - mo0

    def const3(z, x0, Q):
        X = z1calc(prob, x0 + Q @ z, z0)
        return 0.5 * np.transpose(X) @ L @ X - 0.5 * np.transpose(X) @ M @ X - e0

    def jac1(z, x0, Q):
        return np.transpose(omega) @ dz1calc(prob, Q, z0)

    def jac2(z, x0, Q):
        X = z1calc(prob, x0 + Q @ z, z0)
        return np.transpose(X) @ M @ dz1calc(prob, Q, z0)

    def jac3(z, x0, Q):
        X = z1calc(prob, x0 + Q @ z, z0)
        dX = dz1calc(prob, Q, z0)
        return np.transpose(X) @ L @ dX - np.transpose(X) @ M @ dX

    return [{"func": const1, "jac": jac1}, {"func": const2, "jac": jac2}, {"func": const3, "jac": jac3}]


def constraints(dic, prob, lift=True):
    if not lift:
        return dict_constraints(dic, prob)
    key = [prob.dt] + list(np.asarray(prob.butcher_tableau.b).ravel())
    return derived([dic["M"], dic["L"], dic["z0"]], ["lkdvRK"] + key, lambda: _lift(dic, prob))


def cgmresWrapper(dic, x0, k, prob=None, pre=None, tol=1e-50, contol=10, lift=True):
    if prob is None:
        raise ValueError("lkdvRK constraints need `prob` (dt and the Butcher weights), as in the reference")
    conlist = constraints(dic, prob, lift)
    if tol > 1e-20:  # lkdvRK/LinearSolver.py:82
        return solvers.cgmres(A=dic["A"], b=dic["b"], x0=x0, k=k, pre=pre, tol=tol, contol=contol, conlist=conlist)
    return solvers.cgmres_p(A=dic["A"], b=dic["b"], x0=x0, k=k, pre=pre, conlist=conlist)


def gmresWrapper(dic, x0, k, tol=1e-50, pre=None, contol=None, prob=None):
    return solvers.gmres(A=dic["A"], b=dic["b"], x0=x0, k=k, tol=tol, pre=pre)


def exact(dic, x0, k=None, tol=None, prob=None, pre=None, contol=None):
    """Direct solve (``lkdvRK/LinearSolver.py:105-112``), SciPy on the host."""
    return sps.linalg.spsolve(dic["A"], dic["b"]), -1
