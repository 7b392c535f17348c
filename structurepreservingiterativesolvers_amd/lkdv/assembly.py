"""Synthetic assembly of the linear KdV problem (reference ``lkdv/lkdv.py``).

Exact 1-D DG(1) element algebra on ``PeriodicIntervalMesh(M, 40)``
(``lkdv/lkdv.py:17,23``), mixed space (u, v, w) laid out field-major
(``lkdv/refd.py:34-62``; ``np.asarray(...).reshape(-1)``, ``lkdv/lkdv.py:111``).

Forms (``lkdv/lkdv.py:59-61,96-105``), with ``g(u, v) = int u' v dx -
sum_facets jump(u, n) avg(v)``:

* ``F1 = (u - u0)/dt phi + g(v, phi)``
* ``F2 = (v - (u + u0)/2) psi - g((w + w0)/2, psi)``
* ``F3 = w chi - g(u, chi)``

Sparsity follows Firedrake/PyOP2: a block that carries an interior-facet
integral couples every dof of both facet cells (explicit zeros included), so
u/v/w rows carry 8/10/8 entries (8.67 nnz per row on average).

Everything here is exact element algebra except the initial condition, which
is the DG(1) L2 projection of ``sin(beta x) + 1`` computed by 2-point Gauss
quadrature per cell (Firedrake projects with a higher-order rule).
"""
from __future__ import annotations

import numpy as np

from .._assembly import Triplets, embed_blocks, with_pattern


class problem:
    """Mirror of ``lkdv/lkdv.py:15-37``."""

    def __init__(self, N, M, degree, space="DG"):
        if int(degree) < 1 or space != "DG":
            raise NotImplementedError("synthetic lkdv assembly supports DG(q), q >= 1")
        self.mlength = 40
        self.degree = degree
        self.dim = 3
        self.N = N
        self.M = M
        self.space = space
        self.h = self.mlength / M

    def exact(self, x, t):
        alpha = 4
        period = 2 * np.pi / self.mlength
        beta = alpha * period
        return np.sin(beta * (x - (1 - beta ** 2) * t)) + 1


def dg1_operators(M, length):
    """DG(1) mass and ``g`` on a periodic interval: returns (Mass, G, Gpat).

    ``G[i, j] = g(phi_j, phi_i)``; ``Gpat`` is the cell+facet sparsity pattern
    (zeros) that any block carrying ``g`` has.
    """
    h = length / M
    n = 2 * M
    cells = np.arange(M)
    cdofs = np.stack([2 * cells, 2 * cells + 1], axis=1)
    mass_e = np.broadcast_to(h / 6.0 * np.array([[2.0, 1.0], [1.0, 2.0]]), (M, 2, 2))
    Mass = Triplets(n, n).add_blocks(cdofs, cdofs, mass_e).csr()

    # volume term  int phi_j' phi_i = (+-1/h)(h/2)
    vol = np.broadcast_to(np.array([[-0.5, 0.5], [-0.5, 0.5]]), (M, 2, 2))
    t = Triplets(n, n).add_blocks(cdofs, cdofs, vol)
    # facet f sits between L = f-1 (its dof 1) and R = f (its dof 0), periodic.
    left = (cells - 1) % M
    fdofs = np.stack([2 * left, 2 * left + 1, 2 * cells, 2 * cells + 1], axis=1)
    # -(u_L1 - u_R0) * (v_L1 + v_R0)/2 ; local order (L0, L1, R0, R1)
    fac = np.zeros((4, 4))
    for test in (1, 2):
        fac[test, 1] += -0.5
        fac[test, 2] += +0.5
    t.add_blocks(fdofs, fdofs, np.broadcast_to(fac, (M, 4, 4)))
    G = t.csr()
    Gpat = Triplets(n, n).add_blocks(fdofs, fdofs, np.zeros((M, 4, 4))).csr()
    return Mass, G, Gpat, cdofs


def _lagrange(q):
    """Equispaced Lagrange basis of degree q on [0, 1] (nodes include both ends, so a facet value
    is one dof of each cell, as in DG(1)): the monomial coefficients C, phi_j = sum_k C[k, j] x^k."""
    nodes = np.linspace(0.0, 1.0, q + 1)
    return np.linalg.inv(np.vander(nodes, q + 1, increasing=True))


def _basis(C, x, deriv=False):
    """phi_j(x) (or phi_j'(x)) for every j, as (q + 1, len(x))."""
    q = C.shape[0] - 1
    if deriv:
        P = np.zeros((len(x), q + 1))
        for k in range(1, q + 1):
            P[:, k] = k * x ** (k - 1)
    else:
        P = np.vander(x, q + 1, increasing=True)
    return (P @ C).T


def _gauss01(npts):
    xg, wg = np.polynomial.legendre.leggauss(npts)
    return 0.5 * (xg + 1.0), 0.5 * wg


def dg_operators(M, length, q=1):
    """DG(q) mass and ``g`` on a periodic interval (exact Gauss quadrature): (Mass, G, Gpat,
    cdofs).  q = 1 is :func:`dg1_operators` itself (the golden fixtures were made from it; the
    general code at q = 1 agrees with it to rounding, tests/test_assembly_dgq.py)."""
    if q == 1:
        return dg1_operators(M, length)
    return _dg_operators_general(M, length, q)


def _dg_operators_general(M, length, q):
    """dg_operators' element algebra for any q >= 1 (Lagrange basis on equispaced nodes)."""
    h = length / M
    nl = q + 1
    n = nl * M
    cells = np.arange(M)
    cdofs = nl * cells[:, None] + np.arange(nl)[None, :]
    C = _lagrange(q)
    xg, wg = _gauss01(q + 1)  # exact for the degree-2q mass and degree-(2q-1) volume integrands
    phi, dphi = _basis(C, xg), _basis(C, xg, deriv=True)
    mass_e = h * (phi * wg) @ phi.T
    vol_e = (phi * wg) @ dphi.T  # [i, j] = int phi_j' phi_i dx (h cancels)
    Mass = Triplets(n, n).add_blocks(cdofs, cdofs, np.broadcast_to(mass_e, (M, nl, nl))).csr()
    t = Triplets(n, n).add_blocks(cdofs, cdofs, np.broadcast_to(vol_e, (M, nl, nl)))
    # facet between L = cell - 1 (its last dof: u_L(1)) and R = cell (its first dof: u_R(0)):
    # -(u_L(1) - u_R(0)) * (v_L(1) + v_R(0)) / 2, local order (L_0 .. L_q, R_0 .. R_q)
    left = (cells - 1) % M
    fdofs = np.concatenate([cdofs[left], cdofs], axis=1)
    fac = np.zeros((2 * nl, 2 * nl))
    for test in (q, q + 1):
        fac[test, q] += -0.5
        fac[test, q + 1] += +0.5
    t.add_blocks(fdofs, fdofs, np.broadcast_to(fac, (M, 2 * nl, 2 * nl)))
    G = t.csr()
    Gpat = Triplets(n, n).add_blocks(fdofs, fdofs, np.zeros((M, 2 * nl, 2 * nl))).csr()
    return Mass, G, Gpat, cdofs


def project_dg(f, M, length, q=1):
    """L2 projection of ``f`` into DG(q) (q + 2 Gauss points per cell); q = 1 is
    :func:`project_dg1`."""
    if q == 1:
        return project_dg1(f, M, length)
    return _project_dg_general(f, M, length, q)


def _project_dg_general(f, M, length, q):
    h = length / M
    C = _lagrange(q)
    xg, wg = _gauss01(q + 2)
    x0 = np.arange(M)[:, None] * h
    fq = f(x0 + xg[None, :] * h)  # (M, npts)
    phi = _basis(C, xg)  # (q + 1, npts)
    rhs = h * (fq * wg) @ phi.T  # (M, q + 1)
    mass_e = h * (_basis(C, _gauss01(q + 1)[0]) * _gauss01(q + 1)[1]) @ _basis(C, _gauss01(q + 1)[0]).T
    return np.linalg.solve(mass_e, rhs.T).T.reshape(-1)


def project_dg1(f, M, length):
    """L2 projection of ``f`` into DG(1) (2-point Gauss per cell; the DG mass
    matrix is block-diagonal so this is exact for the quadrature)."""
    h = length / M
    xi = np.array([0.5 - 0.5 / np.sqrt(3.0), 0.5 + 0.5 / np.sqrt(3.0)])
    x0 = np.arange(M)[:, None] * h
    xq = x0 + xi[None, :] * h
    fq = f(xq)  # (M, 2)
    phi = np.stack([1 - xi, xi], axis=0)  # phi[i, q]
    rhs = 0.5 * h * fq @ phi.T  # (M, 2)
    minv = np.linalg.inv(h / 6.0 * np.array([[2.0, 1.0], [1.0, 2.0]]))
    return (rhs @ minv.T).reshape(-1)


def solve_mass(Mass, rhs, q=1):
    """Mass^{-1} rhs for the block-diagonal DG(q) mass ((q + 1) x (q + 1) blocks)."""
    if q != 1:
        nl = q + 1
        blk = Mass[:nl, :nl].toarray()  # uniform mesh: every cell's block is the same
        return np.linalg.solve(blk, np.asarray(rhs).reshape(-1, nl).T).T.reshape(-1)
    d = Mass.diagonal()
    off = np.asarray(Mass[np.arange(0, Mass.shape[0], 2), np.arange(1, Mass.shape[0], 2)]).ravel()
    a, bb = d[0::2], d[1::2]
    det = a * bb - off * off
    r0, r1 = rhs[0::2], rhs[1::2]
    out = np.empty_like(rhs)
    out[0::2] = (bb * r0 - off * r1) / det
    out[1::2] = (a * r1 - off * r0) / det
    return out


def linforms(N=100, M=50, degree=1, T=1, space="DG", zinit=None):
    prob = problem(N=N, M=M, degree=degree, space=space)
    q = int(degree)
    Mass, G, Gpat, _ = dg_operators(M, prob.mlength, q)
    nf = (q + 1) * M
    n = 3 * nf
    off = [0, nf, 2 * nf]
    if zinit is None:
        u0 = project_dg(lambda x: prob.exact(x, 0.0), M, prob.mlength, q)
        w0 = solve_mass(Mass, G @ u0, q)  # gfuncproject, lkdv/lkdv.py:62-69,79
    else:
        zinit = np.asarray(zinit, dtype=np.float64)
        u0, w0 = zinit[:nf].copy(), zinit[2 * nf:].copy()
    dt = float(T) / N
    Gf = with_pattern(G, Gpat)
    A = embed_blocks(
        {
            (0, 0): Mass * (1.0 / dt),
            (0, 1): Gf,
            (1, 0): Mass * -0.5,
            (1, 1): Mass,
            (1, 2): Gf * -0.5,
            (2, 0): Gf * -1.0,
            (2, 2): Mass,
        },
        off,
        n,
    )
    b = np.zeros(n)
    b[:nf] = Mass @ u0 / dt
    b[nf:2 * nf] = 0.5 * (Mass @ u0) + 0.5 * (G @ w0)
    Mfull = embed_blocks({(0, 0): Mass}, off, n)
    Lfull = embed_blocks({(2, 2): Mass}, off, n)
    omega = np.zeros(n)
    omega[:nf] = np.asarray(Mass.sum(axis=0)).ravel()
    z_vec = np.zeros(n)
    z_vec[:nf] = u0
    z_vec[2 * nf:] = w0
    out = {
        "A": A,
        "b": b,
        "z0": z_vec,
        "M": Mfull,
        "L": Lfull,
        "omega": omega,
        "m0": float(omega[:nf] @ u0),
        "mo0": float(0.5 * u0 @ Mass @ u0),
        "e0": float(0.5 * w0 @ Mass @ w0 - 0.5 * u0 @ Mass @ u0),
        "T": T,
        "_step": {"Mass": Mass, "G": G, "dt": dt, "nf": nf},  # for step_forms
    }
    return out, prob


def step_forms(dic, zinit):
    """``linforms(..., zinit=z)`` for the next time step (``lkdv/Evolve.py:41``) without
    rebuilding the operators: ``A``, ``M``, ``L``, ``omega`` are the same objects (so they stay
    resident in HBM), ``b``, ``z0`` and the invariant targets are recomputed from ``z``."""
    st = dic["_step"]
    Mass, G, dt, nf = st["Mass"], st["G"], st["dt"], st["nf"]
    z = np.asarray(zinit, dtype=np.float64)
    u0, w0 = z[:nf].copy(), z[2 * nf:].copy()
    n = 3 * nf
    b = np.zeros(n)
    b[:nf] = Mass @ u0 / dt
    b[nf:2 * nf] = 0.5 * (Mass @ u0) + 0.5 * (G @ w0)
    z_vec = np.zeros(n)
    z_vec[:nf] = u0
    z_vec[2 * nf:] = w0
    out = dict(dic)
    out.update(b=b, z0=z_vec, m0=float(dic["omega"][:nf] @ u0), mo0=float(0.5 * u0 @ Mass @ u0),
               e0=float(0.5 * w0 @ Mass @ w0 - 0.5 * u0 @ Mass @ u0))
    return out


def compute_invariants(prob, dic, uvec):
    """``lkdv/lkdv.py:154-166`` on the assembled operators."""
    return {
        "mass": float(dic["omega"] @ uvec),
        "momentum": float(0.5 * uvec @ dic["M"] @ uvec),
        "energy": float(0.5 * uvec @ dic["L"] @ uvec - 0.5 * uvec @ dic["M"] @ uvec),
    }
