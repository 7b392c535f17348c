"""Synthetic assembly of the Gauss-Legendre stage system (reference ``lkdvRK/lkdvRK.py``).

The reference writes the linear KdV system as an ODE/DAE ``M_t z' + K z = 0``
(``lkdvRK/lkdvRK.py:107-111``; only ``u`` carries a time derivative) and lets
Irksome build the s-stage collocation system in stage-derivative form
(``irk.getForm``, ``:113-118``).  Its Jacobian in the stage unknowns
``zbig = [k_1 .. k_s]`` (stage-major, each field-major, ``lkdvRK/lkdvRK.py:171-172``)
is

    A = I_s (x) M_t + dt (A_GL (x) K),      b = -1_s (x) (K z0),

with ``K = [[0, G, 0], [-Mass, Mass, -G], [-G, 0, Mass]]`` in (u, v, w) and
``G`` the DG ``gfunc`` of ``lkdv`` (shared with :mod:`..lkdv.assembly`).  Every
stage pair carries K's full pattern (A_GL is dense), so rows have
``2 + 6s`` / ``10s`` / ``8s`` entries (24.67 nnz/row at s=3).

Irksome is absent, so the Gauss-Legendre tableau is hard-coded for s = 1, 2, 3.
``z1calc``/``dz1calc`` restate ``lkdvRK/lkdvRK.py:162-189``.
"""
from __future__ import annotations

import copy

import numpy as np

from .._assembly import Triplets, embed_blocks, with_pattern
from ..lkdv.assembly import dg_operators, project_dg, solve_mass


def gauss_legendre(s):
    """Butcher tableau (A, b, c) of the s-stage Gauss-Legendre method."""
    if s == 1:
        return np.array([[0.5]]), np.array([1.0]), np.array([0.5])
    if s == 2:
        r = np.sqrt(3.0) / 6.0
        A = np.array([[0.25, 0.25 - r], [0.25 + r, 0.25]])
        return A, np.array([0.5, 0.5]), np.array([0.5 - r, 0.5 + r])
    if s == 3:
        r = np.sqrt(15.0)
        A = np.array(
            [
                [5 / 36, 2 / 9 - r / 15, 5 / 36 - r / 30],
                [5 / 36 + r / 24, 2 / 9, 5 / 36 - r / 24],
                [5 / 36 + r / 30, 2 / 9 + r / 15, 5 / 36],
            ]
        )
        return A, np.array([5 / 18, 4 / 9, 5 / 18]), np.array([0.5 - r / 10, 0.5, 0.5 + r / 10])
    raise NotImplementedError("Gauss-Legendre tableau hard-coded for s <= 3 (Irksome absent)")


class _Tableau:
    def __init__(self, s):
        self.A, self.b, self.c = gauss_legendre(s)
        self.num_stages = s


class problem:
    """Mirror of ``lkdvRK/lkdvRK.py:16-46``."""

    def __init__(self, N, M, degree, tstages, space="DG", T=1):
        if int(degree) < 1 or space != "DG":
            raise NotImplementedError("synthetic lkdvRK assembly supports DG(q), q >= 1")
        self.mlength = 40
        self.degree = degree
        self.tstages = tstages
        self.dim = 3
        self.N = N
        self.M = M
        self.dt = float(T) / N
        self.space = space
        self.butcher_tableau = _Tableau(tstages)
        self.ns = self.butcher_tableau.num_stages
        self.nf = self.dim

    def exact(self, x, t):
        alpha = 4
        period = 2 * np.pi / self.mlength
        beta = alpha * period
        return np.sin(beta * (x - (1 - beta ** 2) * t)) + 1


def linforms(N=100, M=50, degree=1, tstages=2, T=10, t=0.0, zinit=None):
    prob = problem(N=N, M=M, T=T, degree=degree, tstages=tstages)
    q = int(degree)
    Mass, G, Gpat, _ = dg_operators(M, prob.mlength, q)
    nf = (q + 1) * M
    dof = 3 * nf
    s = prob.ns
    n = s * dof
    off3 = [0, nf, 2 * nf]
    if zinit is None:
        u0 = project_dg(lambda x: prob.exact(x, t), M, prob.mlength, q)
        w0 = solve_mass(Mass, G @ u0, q)  # w_finder, lkdvRK/lkdvRK.py:75-82
        v0 = solve_mass(Mass, Mass @ u0 + G @ w0, q)  # v_finder, :64-73
    else:
        zinit = np.asarray(zinit, dtype=np.float64)
        u0, v0, w0 = zinit[:nf].copy(), zinit[nf:2 * nf].copy(), zinit[2 * nf:].copy()
    Gf = with_pattern(G, Gpat)
    K = embed_blocks(
        {
            (0, 1): Gf,
            (1, 0): Mass * -1.0,
            (1, 1): Mass,
            (1, 2): Gf * -1.0,
            (2, 0): Gf * -1.0,
            (2, 2): Mass,
        },
        off3,
        dof,
    )
    Mt = embed_blocks({(0, 0): Mass}, off3, dof)
    Agl, _, _ = gauss_legendre(s)
    dt = prob.dt
    t3 = Triplets(n, n)
    for i in range(s):
        for j in range(s):
            t3.add_csr(K, i * dof, j * dof, scale=dt * Agl[i, j])
        t3.add_csr(Mt, i * dof, i * dof)
    A = t3.csr()
    z0 = np.concatenate([u0, v0, w0])
    Kz0 = K @ z0
    b = -np.tile(Kz0, s)
    out = {
        "A": A,
        "b": b,
        "M": Mt,
        "L": embed_blocks({(2, 2): Mass}, off3, dof),
        "omega": np.concatenate([np.asarray(Mass.sum(axis=0)).ravel(), np.zeros(2 * nf)]),
        "m0": float(np.asarray(Mass.sum(axis=0)).ravel() @ u0),
        "mo0": float(0.5 * u0 @ Mass @ u0),
        "e0": float(0.5 * (w0 @ Mass @ w0 - u0 @ Mass @ u0)),
        "T": T,
        "z0": z0,
        "_step": {"K": K, "Mass": Mass, "s": s, "nf": nf},  # for step_forms
    }
    return out, prob


def step_forms(dic, zinit):
    """``linforms(..., zinit=z)`` for the next time step (``lkdvRK/Evolve.py:55-58``) without
    rebuilding the stage operator (``A``, ``M``, ``L``, ``omega`` stay the same objects)."""
    st = dic["_step"]
    K, Mass, s, nf = st["K"], st["Mass"], st["s"], st["nf"]
    z0 = np.asarray(zinit, dtype=np.float64).copy()
    u0, w0 = z0[:nf], z0[2 * nf:]
    out = dict(dic)
    out.update(b=-np.tile(K @ z0, s), z0=z0, m0=float(dic["omega"][:nf] @ u0), mo0=float(0.5 * u0 @ Mass @ u0),
               e0=float(0.5 * (w0 @ Mass @ w0 - u0 @ Mass @ u0)))
    return out


def z1calc(prob, zbig, z0):
    """``lkdvRK/lkdvRK.py:162-174``: z1 = z0 + dt sum_s b_s zbig[s*dof:(s+1)*dof]."""
    dt = prob.dt
    b = prob.butcher_tableau.b
    dof = len(z0)
    z1 = copy.deepcopy(z0)
    for s in range(prob.ns):
        z1 += dt * b[s] * zbig[s * dof:(s + 1) * dof]
    return z1


def dz1calc(prob, Q, z0):
    """``lkdvRK/lkdvRK.py:178-189``: Jacobian of z1calc w.r.t. zbig applied to Q."""
    dt = prob.dt
    b = prob.butcher_tableau.b
    dof = len(z0)
    dz1 = np.zeros((len(z0), np.shape(Q)[-1]))
    for s in range(prob.ns):
        dz1 += dt * b[s] * Q[s * dof:(s + 1) * dof, :]
    return dz1


def compute_invariants(prob, dic, zbig):
    """Invariants of z1 = z1calc(zbig) on the assembled single-stage operators."""
    z1 = z1calc(prob, zbig, dic["z0"])
    return {
        "mass": float(dic["omega"] @ z1),
        "momentum": float(0.5 * z1 @ dic["M"] @ z1),
        "energy": float(0.5 * z1 @ dic["L"] @ z1 - 0.5 * z1 @ dic["M"] @ z1),
    }
