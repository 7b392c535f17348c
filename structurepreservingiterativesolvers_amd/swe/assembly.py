"""Synthetic shallow-water-shaped system (reference ``swe/swe.py``).

The reference discretises linear rotating shallow water with RT2 x DG0 on a
``PeriodicSquareMesh(M, M, 40)`` (``swe/swe.py:26-32``) and implicit midpoint
in time (``:75-86``).  Firedrake is absent, so this module builds an operator
with the same dof layout, sparsity and conservation structure, but synthetic
element values:

* mesh: 2 M^2 triangles, 3 M^2 periodic edges; RT2 carries 2 dofs per edge
  and 2 interior dofs per cell, DG0 one dof per cell, so N = 12 M^2,
  field-major ``[u (10 M^2) | rho (2 M^2)]`` (``swe/refd.py:36-67``);
* per cell, 9 local dofs; edge-dof rows couple two cells (16 nnz), interior
  RT and DG0 rows one cell (9 nnz): 12.5 nnz per row;
* cell blocks (seeded): ``Mu`` random SPD (RT mass), ``S`` random skew
  (Coriolis ``f (-u_y, u_x)``), ``d`` the flux-divergence weights
  (``+-w_e`` on the two cells of an edge, 0 on interior dofs, so
  ``sum_c d_c = 0`` exactly like ``int div u = 0`` on a periodic mesh),
  ``m`` = cell area (DG0 mass);
* ``A_c = [[Mu/dt + f S/2, -c^2 d/2], [d'/2, m/dt]]`` (lhs of ``F1 + F2``),
  ``b = B z0`` with ``B_c = [[Mu/dt - f S/2, c^2 d/2], [-d'/2, m/dt]]``;
* ``L = blockdiag(Mu, c^2 m)`` (energy, ``swe/swe.py:95``),
  ``omega = int psi`` (``:99``), ``m0 = omega . z0``, ``e0 = 1/2 z0' L z0``.

Because ``d`` has zero column sums and ``[[f S, -c^2 d], [c^2 d', 0]]`` is
skew, the exact solution of ``A z = b`` conserves mass and energy, as the
reference discretisation does — so the constraint projection of CGMRES sees
a consistent (feasible) problem, as in the paper's experiments.
"""
from __future__ import annotations

import numpy as np

from .._assembly import Triplets


class problem:
    """Mirror of ``swe/swe.py:14-40`` (mesh replaced by index arrays)."""

    def __init__(self, N, M, degree, T, seed=0):
        self.mlength = 40
        self.degree = degree
        self.c = 1
        self.f = 0.1
        self.N = N
        self.M = M
        self.T = T
        self.dt = float(T) / N
        self.seed = seed

    def ic(self, x, y):
        u = (0.0, 0.0)
        rho = 10 * np.exp(-((x - 20) ** 2 + (y - 20) ** 2) / 20 ** 2)
        return u, rho


def mesh_topology(M):
    """Periodic M x M square mesh split into 2 M^2 triangles.

    Returns ``cell_edges`` (2M^2, 3) global edge ids, ``cell_sign`` (2M^2, 3)
    orientation (+1 for the first cell that lists an edge, -1 for the second)
    and cell centroids (unit = one square).
    """
    i, j = np.meshgrid(np.arange(M), np.arange(M), indexing="xy")
    i, j = i.ravel(), j.ravel()
    sq = i + M * j
    ip = (i + 1) % M + M * j
    jp = i + M * ((j + 1) % M)
    eh = lambda s: 3 * s + 0  # noqa: E731  horizontal edge of square s
    ev = lambda s: 3 * s + 1  # noqa: E731  vertical edge
    ed = lambda s: 3 * s + 2  # noqa: E731  diagonal
    lower = np.stack([eh(sq), ev(ip), ed(sq)], axis=1)
    upper = np.stack([ed(sq), eh(jp), ev(sq)], axis=1)
    cell_edges = np.empty((2 * M * M, 3), dtype=np.int64)
    cell_edges[0::2] = lower
    cell_edges[1::2] = upper
    # orientation: +1 for the first occurrence of an edge in cell order
    flat = cell_edges.ravel()
    order = np.argsort(flat, kind="stable")
    first = np.zeros(flat.size, dtype=bool)
    first[order[0::2]] = True
    cell_sign = np.where(first, 1.0, -1.0).reshape(cell_edges.shape)
    cx = np.empty(2 * M * M)
    cy = np.empty(2 * M * M)
    cx[0::2], cy[0::2] = i + 2.0 / 3.0, j + 1.0 / 3.0
    cx[1::2], cy[1::2] = i + 1.0 / 3.0, j + 2.0 / 3.0
    return cell_edges, cell_sign, cx, cy


def linforms(N=100, M=50, degree=1, T=10, zinit=None, seed=0):
    prob = problem(N=N, M=M, degree=degree, T=T, seed=seed)
    rng = np.random.default_rng(seed)
    cell_edges, cell_sign, cx, cy = mesh_topology(M)
    nc = 2 * M * M
    ne = 3 * M * M
    nu = 2 * ne + 2 * nc  # = 10 M^2
    n = nu + nc  # = 12 M^2
    hx = prob.mlength / M
    area = 0.5 * hx * hx
    # local dofs: 3 edges x 2, 2 interior, 1 rho
    ldofs = np.empty((nc, 9), dtype=np.int64)
    ldofs[:, 0:6:2] = 2 * cell_edges
    ldofs[:, 1:6:2] = 2 * cell_edges + 1
    ldofs[:, 6] = 2 * ne + 2 * np.arange(nc)
    ldofs[:, 7] = ldofs[:, 6] + 1
    ldofs[:, 8] = nu + np.arange(nc)

    B8 = rng.normal(scale=0.3, size=(nc, 8, 8))
    Mu = area * (0.5 * np.eye(8)[None] + np.einsum("cik,cjk->cij", B8, B8) / 8.0)
    C8 = rng.normal(scale=0.1, size=(nc, 8, 8))
    S = area * (C8 - np.transpose(C8, (0, 2, 1)))
    w_edge = 0.5 * hx * (1.0 + 0.2 * rng.random((ne, 2)))
    d = np.zeros((nc, 8))
    d[:, 0:6:2] = cell_sign * w_edge[cell_edges, 0]
    d[:, 1:6:2] = cell_sign * w_edge[cell_edges, 1]
    dt, f, c2 = prob.dt, prob.f, prob.c ** 2

    Ae = np.zeros((nc, 9, 9))
    Ae[:, :8, :8] = Mu / dt + 0.5 * f * S
    Ae[:, :8, 8] = -0.5 * c2 * d
    Ae[:, 8, :8] = 0.5 * d
    Ae[:, 8, 8] = area / dt
    A = Triplets(n, n).add_blocks(ldofs, ldofs, Ae).csr()
    Be = Ae.copy()
    Be[:, :8, :8] = Mu / dt - 0.5 * f * S
    Be[:, :8, 8] = 0.5 * c2 * d
    Be[:, 8, :8] = -0.5 * d
    del Ae
    Bop = Triplets(n, n).add_blocks(ldofs, ldofs, Be).csr()
    del Be
    L = (
        Triplets(n, n)
        .add_blocks(ldofs[:, :8], ldofs[:, :8], Mu)
        .add_blocks(ldofs[:, 8:], ldofs[:, 8:], np.full((nc, 1, 1), c2 * area))
        .csr()
    )
    if zinit is None:
        z0 = np.zeros(n)
        z0[nu:] = prob.ic(cx * hx, cy * hx)[1]
    else:
        z0 = np.asarray(zinit, dtype=np.float64).copy()
    omega = np.zeros(n)
    omega[nu:] = area
    out = {
        "A": A,
        "b": Bop @ z0,
        "omega": omega,
        "L": L,
        "m0": float(omega @ z0),
        "e0": float(0.5 * z0 @ L @ z0),
        "z0": z0,
        "T": T,
        "_step": {"B": Bop},  # for step_forms
    }
    return out, prob


def step_forms(dic, zinit):
    """``linforms(..., zinit=z)`` for the next time step (``swe/Evolve.py:40``) without
    rebuilding the operators (``A``, ``L``, ``omega`` are the same objects, resident in HBM)."""
    z0 = np.asarray(zinit, dtype=np.float64).copy()
    out = dict(dic)
    out.update(b=dic["_step"]["B"] @ z0, z0=z0, m0=float(dic["omega"] @ z0), e0=float(0.5 * z0 @ dic["L"] @ z0))
    return out


def extra_constraint(n, z_ref, seed=2):
    """Third synthetic quadratic constraint for config C5: a
    random SPD diagonal ``D`` with ``c = -1/2 z_ref' D z_ref`` (swe itself has
    only mass and energy, ``swe/LinearSolver.py:36``)."""
    import scipy.sparse as sps

    rng = np.random.default_rng(seed)
    dg = 0.5 + rng.random(n)
    D = sps.diags(dg, format="csr")
    from .._assembly import to_petsc_csr

    return to_petsc_csr(D), -0.5 * float(z_ref @ (dg * z_ref))


def compute_invariants(prob, dic, vec):
    """``swe/swe.py:121-133`` on the assembled operators."""
    return {"mass": float(dic["omega"] @ vec), "energy": float(0.5 * vec @ dic["L"] @ vec)}
