"""Synthetic assembly of the heat problem (reference ``heat/heat.py``).

Restates ``heat/heat.py:35-121`` without Firedrake: continuous P1 on the
``UnitSquareMesh(M, M)`` (``heat/heat.py:23``, 2-D, N = (M+1)^2), implicit
midpoint in time (``:68-72``), so

* ``A = Mass/dt + 1/2 K``             (lhs of ``F``, ``:71-77``)
* ``b = Mass z0/dt - 1/2 K z0``       (rhs of ``F``, ``:78``)
* ``M = Mass``, ``L = K``             (``:82-89``)
* ``Lz0 = K z0``                      (``:92-93``)
* ``old_energy = 1/2 z0'M z0 - 1/4 dt z0'K z0``  (``:96``)
* ``omega = int(phi)``, ``m0 = int(z0)``, ``e0 = 0``  (``:99-103``)

The initial condition ``1e3((x(x-1))^5 + (y(y-1))^6)`` (``:30-32``) is
interpolated at the vertices rather than L2-projected (no mass solve) — the
operators are exact P1 element integrals, the right-hand side is synthetic.
"""
from __future__ import annotations

import numpy as np

from .._assembly import Triplets


class problem:
    """Mirror of ``heat/heat.py:16-32`` (mesh replaced by vertex/cell arrays)."""

    def __init__(self, N, M, degree, T):
        if degree != 1:
            raise NotImplementedError("synthetic heat assembly supports P1 only")
        self.degree = degree
        self.N = N
        self.M = M
        self.T = T
        self.dt = float(T) / N
        n1 = M + 1
        ii, jj = np.meshgrid(np.arange(n1), np.arange(n1), indexing="xy")
        self.coords = np.stack([ii.ravel() / M, jj.ravel() / M], axis=1)
        cells = []
        for j in range(M):
            for i in range(M):
                v00 = i + n1 * j
                v10, v01, v11 = v00 + 1, v00 + n1, v00 + n1 + 1
                cells.append((v00, v10, v11))
                cells.append((v00, v11, v01))
        self.cells = np.asarray(cells, dtype=np.int64)

    def ic(self, x, y):
        return 1e3 * ((x * (x - 1)) ** 5 + (y * (y - 1)) ** 6)


def p1_element_matrices(coords, cells):
    """Exact P1 mass and stiffness element matrices on triangles."""
    p = coords[cells]  # (E, 3, 2)
    x, y = p[..., 0], p[..., 1]
    b = np.stack([y[:, 1] - y[:, 2], y[:, 2] - y[:, 0], y[:, 0] - y[:, 1]], axis=1)
    c = np.stack([x[:, 2] - x[:, 1], x[:, 0] - x[:, 2], x[:, 1] - x[:, 0]], axis=1)
    area = 0.5 * np.abs(b[:, 0] * c[:, 1] - b[:, 1] * c[:, 0])
    mref = (np.ones((3, 3)) + np.eye(3)) / 12.0
    mass = area[:, None, None] * mref[None]
    stiff = (b[:, :, None] * b[:, None, :] + c[:, :, None] * c[:, None, :]) / (4.0 * area[:, None, None])
    return mass, stiff, area


def linforms(N=100, M=50, degree=1, T=10, zinit=None):
    prob = problem(N=N, M=M, degree=degree, T=T)
    n = prob.coords.shape[0]
    mass_e, stiff_e, area = p1_element_matrices(prob.coords, prob.cells)
    Mass = Triplets(n, n).add_blocks(prob.cells, prob.cells, mass_e).csr()
    K = Triplets(n, n).add_blocks(prob.cells, prob.cells, stiff_e).csr()
    if zinit is None:
        z0 = prob.ic(prob.coords[:, 0], prob.coords[:, 1])
    else:
        z0 = np.asarray(zinit, dtype=np.float64).copy()
    dt = prob.dt
    A = Triplets(n, n).add_csr(Mass, scale=1.0 / dt).add_csr(K, scale=0.5).csr()
    b = Mass @ z0 / dt - 0.5 * (K @ z0)
    omega = np.zeros(n)
    np.add.at(omega, prob.cells.ravel(), np.repeat(area / 3.0, 3))
    Lz0 = K @ z0
    old_energy = 0.5 * z0 @ Mass @ z0 - 0.25 * dt * z0 @ K @ z0
    out = {
        "A": A,
        "b": b,
        "M": Mass,
        "Lz0": Lz0,
        "old_energy": old_energy,
        "omega": omega,
        "L": K,
        "m0": float(omega @ z0),
        "e0": 0,
        "z0": z0,
        "dt": dt,
    }
    return out, prob


def compute_invariants(prob, dic, uvec, uold):
    """``heat/heat.py:124-146`` on the assembled operators: mass = int(z),
    energy = 1/2|z|^2_M - 1/2|z_old|^2_M + dt |grad zmid|^2."""
    Mass, K = dic["M"], dic["L"]
    zmid = 0.5 * (uvec + uold)
    return {
        "mass": float(dic["omega"] @ uvec),
        "energy": float(0.5 * uvec @ Mass @ uvec - 0.5 * uold @ Mass @ uold + prob.dt * zmid @ K @ zmid),
    }
