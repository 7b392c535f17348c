"""CSR ingestion from ``.npz`` files: the data format on the caller's side of the hot path.

The reference gets its operators from Firedrake/PETSc (``getValuesCSR`` → ``csr_matrix``,
e.g. ``heat/heat.py``, ``lkdv/lkdv.py``), which is absent here.  A user with the reference's
stack exports a problem dict once (``save_forms``, or ``scipy.sparse.save_npz`` for one
matrix) and runs the solvers here on it (``load_forms`` / ``load_csr``).  Files are read with
``numpy.load(allow_pickle=False)``: nothing in a file is executed.

Layout of a forms bundle: a matrix ``name`` is four arrays ``name@data``, ``name@indices``,
``name@indptr``, ``name@shape``; arrays and scalars are stored under their key; one level of
nested dicts (the assemblies' private ``_step`` operators) uses ``outer.inner`` keys.
Loaded matrices are canonical CSR (sorted int32 indices, float64 data, explicit zeros kept),
the form the device upload expects.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sps

from ._assembly import to_petsc_csr

_PARTS = ("data", "indices", "indptr", "shape")


def _check_csr(data, indices, indptr, shape, name):
    shape = tuple(int(v) for v in np.asarray(shape).ravel())
    if len(shape) != 2 or min(shape) < 0:
        raise ValueError(f"{name}: bad shape {shape}")
    indptr = np.asarray(indptr)
    indices = np.asarray(indices)
    data = np.asarray(data)
    if indptr.ndim != 1 or len(indptr) != shape[0] + 1:
        raise ValueError(f"{name}: indptr has {len(indptr)} entries for {shape[0]} rows")
    if indptr[0] != 0 or np.any(np.diff(indptr) < 0) or indptr[-1] != len(indices) or len(data) != len(indices):
        raise ValueError(f"{name}: inconsistent indptr / indices / data")
    if len(indices) and (indices.min() < 0 or indices.max() >= shape[1]):
        raise ValueError(f"{name}: column index out of range")
    if not np.issubdtype(data.dtype, np.floating) and not np.issubdtype(data.dtype, np.integer):
        raise ValueError(f"{name}: data dtype {data.dtype} is not numeric")
    m = sps.csr_matrix((data.astype(np.float64), indices.astype(np.int64), indptr.astype(np.int64)), shape=shape)
    return to_petsc_csr(m)


def _put_csr(out, key, m):
    m = to_petsc_csr(m)
    out[key + "@data"] = m.data
    out[key + "@indices"] = m.indices
    out[key + "@indptr"] = m.indptr
    out[key + "@shape"] = np.asarray(m.shape, dtype=np.int64)


def save_csr(path, m):
    """One matrix as a ``scipy.sparse.save_npz``-compatible file (readable by ``load_csr`` and by
    ``scipy.sparse.load_npz``)."""
    sps.save_npz(path, to_petsc_csr(m), compressed=False)


def load_csr(path):
    """A CSR matrix from a ``scipy.sparse.save_npz`` file or a one-matrix forms bundle."""
    with np.load(path, allow_pickle=False) as f:
        keys = set(f.files)
        if {"data", "indices", "indptr", "shape"} <= keys:
            fmt = f["format"].item() if "format" in keys else b"csr"
            fmt = fmt.decode() if isinstance(fmt, bytes) else str(fmt)
            if fmt not in ("csr", "csc"):
                raise ValueError(f"{path}: unsupported sparse format {fmt!r}")
            data, indices, indptr, shape = (f[p] for p in _PARTS)
            if fmt == "csc":  # CSR of the transpose, transposed back
                t = _check_csr(data, indices, indptr, tuple(np.asarray(shape)[::-1]), str(path))
                return to_petsc_csr(t.T)
            return _check_csr(data, indices, indptr, shape, str(path))
        mats = sorted({k.split("@")[0] for k in keys if "@" in k})
        if len(mats) != 1:
            raise ValueError(f"{path}: expected one matrix, found {mats}")
        return _check_csr(*(f[f"{mats[0]}@{p}"] for p in _PARTS), f"{path}:{mats[0]}")


def save_forms(path, forms):
    """A problem dict (the ``linforms`` output: CSR operators, vectors, scalars) as one ``.npz``."""
    out = {}

    def put(key, v):
        if "@" in key:
            raise ValueError(f"key {key!r} may not contain '@'")
        if sps.issparse(v):
            _put_csr(out, key, v)
        elif isinstance(v, (int, float, np.integer, np.floating, np.ndarray, list, tuple)):
            arr = np.asarray(v)
            if arr.dtype == object:
                raise ValueError(f"{key}: object arrays are not stored")
            out[key] = arr
        else:
            raise ValueError(f"{key}: cannot store a {type(v).__name__}")

    for k, v in forms.items():
        if "." in k:
            raise ValueError(f"key {k!r} may not contain '.'")
        if isinstance(v, dict):
            for k2, v2 in v.items():
                put(f"{k}.{k2}", v2)
        else:
            put(k, v)
    np.savez(path, **out)


def load_forms(path):
    """Inverse of ``save_forms``: matrices come back as canonical CSR, 0-d arrays as Python
    floats/ints (the reference's ``m0``/``e0``/``T`` are scalars)."""
    forms = {}
    with np.load(path, allow_pickle=False) as f:
        keys = list(f.files)
        mats = sorted({k.split("@")[0] for k in keys if "@" in k})
        vals = {}
        for m in mats:
            missing = [p for p in _PARTS if f"{m}@{p}" not in keys]
            if missing:
                raise ValueError(f"{path}: matrix {m} lacks {missing}")
            vals[m] = _check_csr(*(f[f"{m}@{p}"] for p in _PARTS), f"{path}:{m}")
        for k in keys:
            if "@" in k:
                continue
            a = f[k]
            if a.ndim == 0:
                vals[k] = a.item()
            else:
                vals[k] = a
    for k, v in vals.items():
        if "." in k:
            outer, inner = k.split(".", 1)
            forms.setdefault(outer, {})[inner] = v
        else:
            forms[k] = v
    return forms
