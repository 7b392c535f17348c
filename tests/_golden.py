"""Loader for the golden fixtures written by ``tests/golden/make_golden.py``.

Rebuilds the exact inputs the reference saw (CSR operators, b, x0) and the
constraint list in the reference's own form: class objects with ``M, v, c``
(``heat/LinearSolver.py:26-38``, ``lkdv/LinearSolver.py:28-47``,
``swe/LinearSolver.py:23-36``) or, for lkdvRK, the dict-form ``func``/``jac``
pairs of ``lkdvRK/LinearSolver.py:29-79``.
"""
from __future__ import annotations

import ast
import glob
import os
import types

import numpy as np
import scipy.sparse as sps
import scipy.sparse.linalg as spla

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz")))


def _csr(z, prefix):
    shape = tuple(int(s) for s in z[f"{prefix}_shape"])
    return sps.csr_matrix((z[f"{prefix}_data"], z[f"{prefix}_indices"], z[f"{prefix}_indptr"]), shape=shape)


class _Con:
    def __init__(self, M, v, c):
        self.M, self.v, self.c = M, v, c


class Case:
    def __init__(self, name):
        self.name = name
        z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
        self.z = z
        self.meta = ast.literal_eval(str(z["meta"]))
        self.A = _csr(z, "dic_A")
        self.b = z["b"]
        self.x0 = z["x0"]
        self.x_all = z["x_all"]
        self.x_final = z["x_final"]
        self.res = z["res"]
        self.steps = int(z["steps"])
        self.calls_p = z["calls_p"]
        self.calls_ncons = z["calls_ncons"]
        self.calls_msg = [str(m) for m in z["calls_msg"]]
        self.calls_y = z["calls_y"]
        self.fd_warnings = [str(m) for m in z["fd_warnings"]]
        self.py_warnings = [str(m) for m in z["py_warnings"]]
        self.solver = self.meta["solver"]
        self.k = self.meta["k"]
        self.tol = self.meta["tol"]

    def dic(self):
        """The problem dictionary handed to the reference wrapper."""
        out = {}
        for key in self.z.files:
            if not key.startswith("dic_"):
                continue
            base = key[4:]
            for suf in ("_data", "_indices", "_indptr", "_shape"):
                if base.endswith(suf):
                    mat = base[: -len(suf)]
                    if mat not in out:
                        out[mat] = _csr(self.z, "dic_" + mat)
                    break
            else:
                v = self.z[key]
                out[base] = float(v) if v.ndim == 0 else v
        return out

    def prob(self):
        """lkdvRK ``prob`` surrogate: what ``z1calc`` reads (dt, tableau b, ns)."""
        d = self.dic()
        bb = np.asarray(d["butcher_b"])
        return types.SimpleNamespace(dt=d["dt"], ns=len(bb), butcher_tableau=types.SimpleNamespace(b=bb))

    def conlist(self, zero_mass_as_0A=True):
        """Constraint list exactly as the reference wrapper built it."""
        p = self.meta["problem"]
        d = self.dic()
        A = d.get("A")
        zero = (0 * A) if zero_mass_as_0A else sps.csr_matrix(A.shape)
        if self.meta.get("cons") == "none":
            return []
        if p == "heat":
            return [_Con(zero, np.transpose(d["omega"]), -d["m0"]),
                    _Con(d["M"] + 0.5 * d["dt"] * d["L"], 0.5 * d["dt"] * d["Lz0"], -d["old_energy"])]
        if p == "lkdv":
            z0 = np.zeros_like(self.x0)
            return [_Con(zero, np.transpose(d["omega"]), -d["m0"]),
                    _Con(d["M"], np.zeros_like(z0), -d["mo0"]),
                    _Con(d["L"] - d["M"], np.zeros_like(z0), -d["e0"])]
        if p == "swe":
            return [_Con(zero, np.transpose(d["omega"]), -d["m0"]),
                    _Con(d["L"], np.zeros_like(self.x0), -d["e0"])]
        if p == "swe3":
            return [_Con(zero, d["omega"], -d["m0"]),
                    _Con(d["L"], np.zeros_like(self.x0), -d["e0"]),
                    _Con(d["D3"], np.zeros_like(self.x0), d["c3"])]
        if p == "lkdvRK":
            return lkdvrk_dict_constraints(d, self.prob())
        raise KeyError(p)

    def preconditioner(self):
        pre = self.meta.get("pre")
        if pre is None:
            return None
        if pre == "jacobi":
            return sps.diags(1.0 / self.A.diagonal(), format="csr")
        if pre == "spilu":
            return spla.spilu(self.A.tocsc(), drop_tol=1e-2, fill_factor=10)
        raise KeyError(pre)

    def kwargs(self):
        kw = {}
        if "contol" in self.meta:
            kw["contol"] = self.meta["contol"]
        if self.meta.get("timing"):
            kw["timing"] = True
        return kw


def lkdvrk_dict_constraints(d, prob):
    """``lkdvRK/LinearSolver.py:29-79`` restated (dict form, z1calc-based)."""
    from structurepreservingiterativesolvers_amd.lkdvRK.assembly import dz1calc, z1calc

    M, L, omega, z0 = d["M"], d["L"], d["omega"], d["z0"]
    m0, mo0, e0 = d["m0"], d["mo0"], d["e0"]

    def const1(z, x0, Q):
        X = z1calc(prob, x0 + Q @ z, z0)
        return np.transpose(omega) @ X - m0

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


def expected_trace(case):
    """Branch per iteration from the SLSQP call log: 'uncon' (no constraints
    passed), 'con', or 'fallback' (a constrained call followed by an
    unconstrained one for the same p).  For cgmres_p, constraints are
    clist[:j], so 'con' means 'the constrained call was kept'.  With an empty
    conlist the constrained branch also passes zero constraints; it is
    entered at the first j with j == k-1 or res[j-1] <= contol*tol and never
    left (``safety`` is no longer None, ``solvers.py:230``)."""
    out = []
    ps, nc = list(case.calls_p), list(case.calls_ncons)
    nocons = case.meta.get("cons") == "none"
    entered = False
    i = 0
    while i < len(ps):
        p = ps[i]
        j = p - 1
        if i + 1 < len(ps) and ps[i + 1] == p:
            out.append((j, "fallback"))
            i += 2
            continue
        if case.solver == "cgmres_p":
            out.append((j, "con"))
        elif nocons:
            prev = np.linalg.norm(case.b - case.A @ case.x0) if j == 0 else case.res[j - 1]
            entered = entered or j == case.k - 1 or not prev > case.meta.get("contol", 10) * case.tol
            out.append((j, "con" if entered else "uncon"))
        else:
            out.append((j, "con" if nc[i] > 0 else "uncon"))
        i += 1
    return out
