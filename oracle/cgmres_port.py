"""ORACLE (test infrastructure only) — CPU restatement of ``solvers.py``.

Each function restates one routine of the reference ``solvers.py`` with the
same NumPy/SciPy primitives in the same evaluation order, so that on identical
inputs it reproduces the reference's floating-point results (this is checked
against the golden vectors in ``tests/golden``).  Line numbers below refer to
``/root/reference/solvers.py``.

Differences from the reference that do not change results:
* Firedrake's ``warning`` (``solvers.py:5,272,419``) is a logging call; it is
  replaced by ``logging.getLogger("spis.oracle").warning``.
* Optional ``trace`` list: every least-squares solve appends
  ``(j, kind)`` with kind in {"uncon", "con", "fallback"}; it is how the
  tests compare branch sequences.
"""
from __future__ import annotations

import logging
import time as _time
import warnings

import numpy as np
import scipy.optimize as spo
import scipy.sparse as sps

_log = logging.getLogger("spis.oracle")

# SLSQP exit messages that ``solvers.py:280-282`` / ``:427-429`` accept silently
_ACCEPTED = (
    "Optimization terminated successfully",
    "`xtol` termination condition is satisfied.",
    "`gtol` termination condition is satisfied.",
)


def constraint_checker(y, eq_list):
    """``solvers.py:14-18``: signed running max, starting from 0."""
    worst = 0
    for item in eq_list:
        worst = max(worst, item["fun"](y))
    return worst


class ConstraintTerms:
    """``solvers.py:21-53``: quadratic constraint reduced onto ``X = x0 + Z y``.

    Class-like constraints (anything with ``__dict__``) carry ``M, v, c`` and
    are reduced to ``term0 + term1.y + y.term2.y``; dict constraints keep their
    ``func``/``jac`` callables ``(y, x0, Z)``.
    """

    def __init__(self, const, x0, Z):
        if hasattr(const, "__dict__"):
            self.reduced = True
        elif type(const) is dict:
            self.reduced = None
        else:
            raise NotImplementedError("Constraints must be either dictionaries or classes")
        if self.reduced:
            MZ = const.M @ Z
            self.MZ = MZ
            self.term0 = 0.5 * x0 @ const.M @ x0 + const.c + const.v @ x0
            self.term1 = const.v @ Z + x0 @ MZ
            self.term2 = 0.5 * Z.T @ MZ
        else:
            self.const, self.x0, self.Z = const, x0, Z

    def value(self, y):
        if self.reduced:
            return self.term0 + self.term1 @ y + y @ self.term2 @ y
        return self.const["func"](y, self.x0, self.Z)

    def gradient(self, y):
        if self.reduced:
            return self.term1 + 2 * y @ self.term2
        return self.const["jac"](y, self.x0, self.Z)

    def as_slsqp(self):
        return {"type": "eq", "fun": self.value, "jac": self.gradient}


def _preconditioner(pre, n):
    """``solvers.py:149-161`` (same in ``gmres`` ``:61-73``, ``cgmres_p`` ``:337-349``)."""
    if pre is None:
        pre = sps.identity(n)
    if hasattr(pre, "solve"):
        return pre.solve

    def apply(vec):
        try:
            out = pre @ vec
        except Exception:
            raise ValueError("Preconditioner not supported")
        return out

    return apply


class _Arnoldi:
    """Shared Arnoldi/MGS state of the three solvers (``solvers.py:78-102``,
    ``:165-202``, ``:351-377``).  Q and Z are row-major ``(k+1, N)``."""

    def __init__(self, A, b, x0, k, pre):
        self.A, self.b, self.x0, self.k = A, b, x0, k
        self.apply_pre = _preconditioner(pre, len(b))
        r = b - A.dot(x0)
        self.r0 = r
        n = np.size(r)
        self.Q = np.zeros((k + 1, n))
        self.Zb = np.zeros((k + 1, n))
        self.beta = np.linalg.norm(r)
        self.Q[0] = r / self.beta
        self.H = np.zeros((k + 1, k))

    def extend(self, j, stop_on_breakdown=True):
        """One Arnoldi step; returns False on breakdown (``h[j+1,j] == 0``)."""
        Q, H = self.Q, self.H
        self.Zb[j] = np.asarray(self.apply_pre(Q[j]))
        w = np.asarray(self.A @ self.Zb[j])
        for i in range(j + 1):
            H[i, j] = np.dot(Q[i], w)
            w = w - H[i, j] * Q[i]
        H[j + 1, j] = np.linalg.norm(w)
        if H[j + 1, j] != 0:
            Q[j + 1] = w / H[j + 1, j]
            return True
        return False

    def ls_objective(self, j):
        """``solvers.py:204-219``: ||beta e1 - H y||^2 and its gradient."""
        rhs = np.zeros(j + 2)
        rhs[0] = self.beta
        Hj = self.H[: j + 2, : j + 1]

        def func(y):
            F = rhs - Hj @ y
            return np.inner(F, F)

        def jac(y):
            F = rhs - Hj @ y
            return -2 * np.transpose(Hj) @ F

        return rhs, func, jac

    def basis(self, j):
        return np.transpose(self.Zb[: j + 1, :])

    def true_residual(self, xj):
        return np.linalg.norm(self.A.dot(xj) - self.b)


def _breakdown_warning():
    warnings.warn("GMRES broke down, either initial guess is exact or" + " , more likely, something has gone wrong.")


def gmres(A, b, x0, k, tol=1e-50, pre=None):
    """``solvers.py:58-127`` (FGMRES, least squares by ``np.linalg.lstsq``)."""
    st = _Arnoldi(A, b, x0, k, pre)
    xs = [st.r0]
    res = [np.linalg.norm(st.r0)]
    steps = 0
    for j in range(k):
        steps = j + 1
        if not st.extend(j):
            _breakdown_warning()
            break
        rhs = np.zeros(j + 2)
        rhs[0] = st.beta
        Z = st.basis(j)
        yk = np.linalg.lstsq(st.H[: j + 2, : j + 1], rhs, rcond=None)[0]
        xs.append(Z @ yk + x0)
        res.append(st.true_residual(xs[-1]))
        if res[-1] < tol:
            break
    return xs[-1], {"name": "gmres", "x": xs, "res": res[1:], "steps": steps}


def _slsqp(func, y0, jac, cons, ftol):
    return spo.minimize(func, y0, tol=None, jac=jac, constraints=cons, method="SLSQP",
                        options={"ftol": ftol, "maxiter": 1e3})


def cgmres(A, b, x0, k, tol=1e-8, contol=10, conlist=[], pre=None, timing=None, trace=None, diag=None):
    """``solvers.py:131-323`` (constrained FGMRES).

    diag (test diagnostics, optional dict): per constrained step j, the signed checker value of
    SLSQP's solution, each reduced constraint's magnitude at it (|term0| + |term1 y| + |y term2 y|:
    the scale its rounding lives on) and SLSQP's message; no effect on the computation."""
    ctol = 1e-12
    if timing:
        stamps = {"start": _time.time(), "start_iter": [], "end_iter": [],
                  "start_constraints": [], "end_constraints": []}
    st = _Arnoldi(A, b, x0, k, pre)
    safety = None
    xs = [st.r0]
    res = [np.linalg.norm(st.r0)]
    n_con_steps = 0
    steps = 0
    yk = None
    for j in range(k):
        if timing:
            stamps["start_iter"].append(_time.time())
        steps = j + 1
        if not st.extend(j):
            _breakdown_warning()
            break
        _, func, jac = st.ls_objective(j)
        Z = st.basis(j)
        y0 = np.zeros((j + 1,))
        if j != 0:
            y0[:-1] = yk
        eq = []
        if res[-1] > contol * tol and j < k - 1 and safety is None:
            sol = _slsqp(func, y0, jac, [], ctol ** 2)
            if trace is not None:
                trace.append((j, "uncon"))
        else:
            try:
                if timing:
                    n_con_steps += 1
                    stamps["start_constraints"].append(_time.time())
                for const in conlist:
                    eq.append(ConstraintTerms(const, x0, Z).as_slsqp())
                if timing:
                    stamps["end_constraints"].append(_time.time())
                sol = _slsqp(func, y0, jac, eq[:], ctol ** 2)
                if diag is not None:
                    ct = [ConstraintTerms(c, x0, Z) for c in conlist]
                    diag[j] = {"nan": bool(np.isnan(max(sol.x))), "violation": constraint_checker(sol.x, eq),
                               "message": sol.message,
                               "scales": [abs(t.term0) + abs(t.term1 @ sol.x) + abs(sol.x @ t.term2 @ sol.x)
                                          if t.reduced else float("nan") for t in ct]}
                if not timing:
                    if np.isnan(max(sol.x)):
                        raise ValueError
                safety = True
                if not timing:
                    if constraint_checker(sol.x, eq) > ctol:
                        safety = False
                        # the reference formats ``solve.constr_violation`` here, which SciPy's
                        # OptimizeResult does not carry: AttributeError -> except below
                        raise AttributeError("constr_violation")
                if trace is not None:
                    trace.append((j, "con"))
            except Exception:
                _log.warning("Constrained solve failed, defaulted to standard solve for iteration %d." % j
                             + " Problem likely overconstrained, a smaller solver tolerance may be required.")
                sol = _slsqp(func, y0, jac, [], ctol ** 2)
                if trace is not None:
                    trace.append((j, "fallback"))
        if sol.message not in _ACCEPTED:
            warnings.warn("Iteration %d failed with message '%s'" % (j, sol.message), RuntimeWarning)
        yk = sol.x
        xs.append(Z @ yk + x0)
        res.append(st.true_residual(xs[-1]))
        if timing:
            stamps["end_iter"].append(_time.time())
        if res[-1] < tol and safety == True:  # noqa: E712  (reference compares with ==)
            break
    timings = None
    if timing:
        stamps["end"] = _time.time()
        per_iter = np.asarray(stamps["end_iter"]) - np.asarray(stamps["start_iter"])
        uncon = per_iter[:-n_con_steps]
        build = np.asarray(stamps["end_constraints"]) - np.asarray(stamps["start_constraints"])
        con = per_iter[len(uncon):] - build
        timings = {"runtime": stamps["end"] - stamps["start"],
                   "iter_time_unconstrained": np.mean(uncon),
                   "iter_time_constrained": np.mean(con),
                   "constraint_building": np.mean(build),
                   "constrained_steps": n_con_steps}
    return xs[-1], {"name": "cgmres", "x": xs, "res": res[1:], "steps": steps, "timings": timings}


def cgmres_p(A, b, x0, k, conlist=[], pre=None, trace=None):
    """``solvers.py:328-445`` (prototypical CGMRES: constraint i enforced from step i)."""
    st = _Arnoldi(A, b, x0, k, pre)
    xs = [st.r0]
    res = []
    yk = None
    for j in range(k):
        st.extend(j)  # no break on breakdown here (solvers.py:376-377)
        _, func, jac = st.ls_objective(j)
        Z = st.basis(j)
        eq = [ConstraintTerms(const, x0, Z).as_slsqp() for const in conlist]
        y0 = np.zeros((j + 1,))
        if j != 0:
            y0[:-1] = yk
        sol = spo.minimize(func, y0, tol=1e-15, jac=jac, constraints=eq[:j], method="SLSQP",
                           options={"ftol": 1e-20, "maxiter": 1e3})
        kind = "con"
        if np.isnan(max(sol.x)):
            _log.warning("Constrained solve silently failed on iteration %d" % j)
            sol = _slsqp(func, y0, jac, [], 1e-20)
            kind = "fallback"
        if trace is not None:
            trace.append((j, kind))
        if sol.message not in _ACCEPTED:
            warnings.warn("Iteration %d failed with message '%s'" % (j, sol.message), RuntimeWarning)
        yk = sol.x
        xs.append(Z @ yk + x0)
        res.append(st.true_residual(xs[-1]))
    return xs[-1], {"name": "geosolve", "x": xs, "res": res}
