"""Element-by-element sparse assembly helpers for the synthetic test problems.

The reference assembles every operator with Firedrake and reads it back as a
SciPy CSR triple (e.g. ``heat/heat.py:76-77``, ``swe/swe.py:90-91``).  Firedrake
is not available here, so the problem modules of this package assemble the same
operators (or operators of the same shape and sparsity) element by element.
These helpers are the scatter step shared by all of them: local element
matrices are scattered through a local-to-global dof map into COO triplets and
summed into CSR with int32 indices and float64 values, the index/value types
PETSc's ``getValuesCSR`` hands the reference.

Explicit zeros are kept on purpose: Firedrake's sparsity includes every
(test dof, trial dof) pair that shares a cell or an interior facet, whether or
not the integral is non-zero there, and nnz is part of what the SpMV pays for.
SciPy's ``A + B`` drops zeros, so everything here goes through COO
concatenation + ``tocsr()`` (which sums duplicates and keeps zeros).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sps


class Triplets:
    """Accumulates COO triplets; ``csr()`` sums duplicates, keeps zeros."""

    def __init__(self, n_rows, n_cols):
        self.shape = (int(n_rows), int(n_cols))
        self.r, self.c, self.v = [], [], []

    def add_blocks(self, row_dofs, col_dofs, blocks):
        """Scatter ``blocks[e] (r x c)`` through ``row_dofs[e]``, ``col_dofs[e]``."""
        row_dofs = np.asarray(row_dofs)
        col_dofs = np.asarray(col_dofs)
        blocks = np.asarray(blocks, dtype=np.float64)
        shp = blocks.shape
        self.r.append(np.broadcast_to(row_dofs[:, :, None], shp).astype(np.int32).ravel())
        self.c.append(np.broadcast_to(col_dofs[:, None, :], shp).astype(np.int32).ravel())
        self.v.append(blocks.ravel())
        return self

    def add_csr(self, m, row_off=0, col_off=0, scale=1.0):
        coo = sps.coo_matrix(m)
        self.r.append((coo.row.astype(np.int64) + row_off).astype(np.int32))
        self.c.append((coo.col.astype(np.int64) + col_off).astype(np.int32))
        self.v.append(coo.data * scale)
        return self

    def csr(self):
        if not self.r:
            return to_petsc_csr(sps.csr_matrix(self.shape))
        r = np.concatenate(self.r)
        c = np.concatenate(self.c)
        v = np.concatenate(self.v)
        m = sps.coo_matrix((v, (r, c)), shape=self.shape).tocsr()
        return to_petsc_csr(m)


def to_petsc_csr(m):
    """Canonical CSR: sorted column indices, int32 index arrays, float64 data,
    explicit zeros retained (what ``csr_matrix((vals, cols, rowptr))`` built from
    ``getValuesCSR`` looks like in the reference)."""
    if not sps.isspmatrix_csr(m):
        m = sps.csr_matrix(m)
    if m.dtype != np.float64:
        m = m.astype(np.float64)
    if not m.has_canonical_format:
        m.sum_duplicates()  # sorts and sums, keeps explicit zeros
    return sps.csr_matrix(
        (m.data, m.indices.astype(np.int32), m.indptr.astype(np.int32)), shape=m.shape
    )


def with_pattern(m, pattern):
    """Return ``m`` re-expressed on the union of its own pattern and
    ``pattern``'s (explicit zeros where only ``pattern`` has entries)."""
    t = Triplets(*m.shape)
    t.add_csr(m)
    t.add_csr(pattern, scale=0.0)
    return t.csr()


def embed_blocks(blocks, offsets, n):
    """Place CSR sub-blocks ``{(bi, bj): csr}`` of a field-major mixed operator
    into one ``n x n`` CSR (``offsets[f]`` is the first global dof of field f)."""
    t = Triplets(n, n)
    for (bi, bj), m in blocks.items():
        t.add_csr(m, offsets[bi], offsets[bj])
    return t.csr()
