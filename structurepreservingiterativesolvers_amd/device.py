"""Device-side handles: context, HBM-resident CSR matrices and vectors.

The reference hands SciPy CSR matrices and NumPy vectors to ``solvers.cgmres``
on every call (e.g. ``swe/LinearSolver.py:46``) and never mutates them
(``solvers.py:167`` allocates).  This module keeps one HBM copy per matrix
object: uploads are cached on ``id(A)`` guarded by the identity of its three
arrays (``data``/``indices``/``indptr`` buffers, shape, nnz) and dropped when the
SciPy object is garbage collected.  Code that mutates ``A.data`` in place must
call :func:`invalidate`.
"""
from __future__ import annotations

import ctypes as C
import os
import weakref

import numpy as np
import scipy.sparse as sps

from . import _lib

_DOUBLE_P = C.POINTER(C.c_double)
_I32_P = C.POINTER(C.c_int32)


class Context:
    """One HIP device + stream (+ optional RCCL communicator)."""

    def __init__(self, device=0):
        self.L = _lib.lib()
        h = C.c_void_p()
        _lib.check(self.L.spis_context_create(int(device), C.byref(h)), "spis_context_create")
        self.handle = h
        self.device = int(device)
        self.nranks = 1
        self.rank = 0

    def synchronize(self):
        _lib.check(self.L.spis_context_synchronize(self.handle), "spis_context_synchronize")

    def close(self):
        """Destroy the context; device objects still alive become inert (their finalizers
        see the closed context and do nothing)."""
        if self.handle:
            self.L.spis_context_destroy(self.handle)
            self.handle = None


_OPTIONS = {
    "fuse_spmv": (_lib.OPT_FUSE_SPMV, None),
    "generic_gram": (_lib.OPT_GENERIC_GRAM, None),
    "graphs": (_lib.OPT_GRAPHS, None),
    "orthog": (_lib.OPT_ORTHOG, {"mgs": 0, "cgs2": 1}),
    "ell_gram": (_lib.OPT_ELL_GRAM, None),
}


def set_option(name, value, ctx=None):
    """Per-context solver options (``spis_set_option``, include/spis.h):

    * ``fuse_spmv`` (True): true-residual and Arnoldi SpMVs in one launch (bit-identical);
    * ``graphs`` (False): replay captured Arnoldi steps;
    * ``orthog`` ("mgs"): "mgs", the reference's modified Gram-Schmidt, or "cgs2", the
      low-synchronisation option (3 reductions per step; not MGS's rounding);
    * ``generic_gram`` (False): constraint reduction via SpMM + tiled Gram (tests);
    * ``ell_gram`` (True): fused constraint reduction on a sliced-ELL copy of each matrix."""
    ctx = ctx or get_context()
    opt, names = _OPTIONS[name]
    v = names[value] if names is not None else int(bool(value))
    _lib.check(ctx.L.spis_set_option(ctx.handle, opt, v), "spis_set_option")


def _release(ctx, fn_name, handle):
    """Finalizer: release a device object unless its context was already destroyed."""
    if ctx.handle:
        getattr(ctx.L, fn_name)(*([ctx.handle] if fn_name == "spis_free" else []), handle)


_CONTEXTS: dict[int, Context] = {}


def default_device():
    env = os.environ.get("SPIS_DEVICE")
    if env is not None:
        return int(env)
    return 0


def get_context(device=None) -> Context:
    dev = default_device() if device is None else int(device)
    ctx = _CONTEXTS.get(dev)
    if ctx is None:
        ctx = Context(dev)
        _CONTEXTS[dev] = ctx
    return ctx


class DeviceBuffer:
    """Raw HBM allocation (fp64 elements) owned by a context."""

    def __init__(self, ctx: Context, n: int):
        self.ctx = ctx
        self.n = int(n)
        p = C.c_void_p()
        _lib.check(ctx.L.spis_malloc(ctx.handle, 8 * max(self.n, 1), C.byref(p)), "spis_malloc")
        self.ptr = p.value
        self._fin = weakref.finalize(self, _release, ctx, "spis_free", C.c_void_p(self.ptr))

    def upload(self, arr):
        a = np.ascontiguousarray(arr, dtype=np.float64)
        if a.size > self.n:
            raise ValueError("upload larger than buffer")
        _lib.check(self.ctx.L.spis_memcpy_h2d(self.ctx.handle, C.c_void_p(self.ptr), a.ctypes.data_as(C.c_void_p),
                                              8 * a.size), "spis_memcpy_h2d")
        return self

    def download(self, n=None):
        n = self.n if n is None else int(n)
        out = np.empty(n, dtype=np.float64)
        _lib.check(self.ctx.L.spis_memcpy_d2h(self.ctx.handle, out.ctypes.data_as(C.c_void_p),
                                              C.c_void_p(self.ptr), 8 * n), "spis_memcpy_d2h")
        return out


class DeviceVector(DeviceBuffer):
    """An fp64 vector resident in HBM (length ``n``, room for ``capacity``)."""

    def __init__(self, ctx: Context, n: int, capacity: int | None = None):
        super().__init__(ctx, n if capacity is None else max(n, capacity))
        self.n_valid = int(n)

    @classmethod
    def from_host(cls, arr, ctx=None, capacity=None):
        arr = np.ascontiguousarray(arr, dtype=np.float64).reshape(-1)
        ctx = ctx or get_context()
        return cls(ctx, arr.size, capacity).upload(arr)

    def numpy(self):
        return self.download(self.n_valid)

    def __len__(self):
        return self.n_valid

    def __array__(self, dtype=None, copy=None):
        a = self.numpy()
        return a if dtype is None else a.astype(dtype)


class DeviceMatrix:
    """CSR matrix resident in HBM (int32 indices, fp64 values).

    ``halo`` (optional) describes ghost columns for a row-partitioned operator
    (see :mod:`.distributed`)."""

    def __init__(self, ctx: Context, A, halo=None):
        A = _as_csr(A)
        self.ctx = ctx
        self.shape = A.shape
        self.nnz = int(A.nnz)
        h = C.c_void_p()
        halo_p = None
        self._keep = None
        if halo is not None:
            self._keep = halo.ctypes_arrays()
            halo_p = C.byref(halo.desc(self._keep))
        _lib.check(
            ctx.L.spis_csr_upload(
                ctx.handle, A.shape[0], A.shape[1], A.nnz,
                A.indptr.ctypes.data_as(_I32_P), A.indices.ctypes.data_as(_I32_P), A.data.ctypes.data_as(_DOUBLE_P),
                halo_p, C.byref(h),
            ),
            "spis_csr_upload",
        )
        self.handle = h
        self._fin = weakref.finalize(self, _release, ctx, "spis_matrix_destroy", h)
        info = (C.c_int64 * 8)()
        _lib.check(ctx.L.spis_matrix_info(h, info), "spis_matrix_info")
        self.n_blocks = int(info[3])
        self.n_long_rows = int(info[4])
        self.n_ghost = int(info[5])
        self.all_zero = bool(info[6])

    @property
    def n_rows(self):
        return self.shape[0]


def _as_csr(A):
    if not sps.isspmatrix_csr(A) and not isinstance(A, sps.csr_array):
        A = sps.csr_matrix(A)
    data = np.ascontiguousarray(A.data, dtype=np.float64)
    indices = A.indices
    indptr = A.indptr
    if indices.dtype != np.int32 or indptr.dtype != np.int32:
        if A.nnz >= 2 ** 31:
            raise ValueError("nnz >= 2^31 not supported (int32 CSR, as PETSc AIJ)")
        indices = indices.astype(np.int32)
        indptr = indptr.astype(np.int32)
    if data is not A.data or indices is not A.indices or indptr is not A.indptr:
        A = sps.csr_matrix((data, np.ascontiguousarray(indices), np.ascontiguousarray(indptr)), shape=A.shape)
    return A


# ---- upload caches --------------------------------------------------------------------------
_MATRIX_CACHE: dict = {}


def _matrix_key(A):
    return (id(A), A.shape, int(A.nnz), A.data.ctypes.data, A.indices.ctypes.data, A.indptr.ctypes.data)


def device_matrix(A, ctx=None) -> DeviceMatrix:
    """HBM copy of SciPy CSR ``A`` (cached for the lifetime of ``A``)."""
    if isinstance(A, DeviceMatrix):
        return A
    ctx = ctx or get_context()
    if not sps.issparse(A):
        return DeviceMatrix(ctx, A)
    key = _matrix_key(A) + (ctx.device,)
    hit = _MATRIX_CACHE.get(key)
    if hit is not None:
        return hit
    dm = DeviceMatrix(ctx, A)
    _MATRIX_CACHE[key] = dm
    try:
        weakref.finalize(A, _MATRIX_CACHE.pop, key, None)
    except TypeError:  # not weak-referenceable: keep until invalidate()
        pass
    return dm


def invalidate(A=None):
    """Forget cached uploads (of ``A``, or all)."""
    if A is None:
        _MATRIX_CACHE.clear()
        return
    for key in [k for k in _MATRIX_CACHE if k[0] == id(A)]:
        _MATRIX_CACHE.pop(key, None)


def device_vector(v, ctx=None, capacity=None) -> DeviceVector:
    if isinstance(v, DeviceVector):
        return v
    return DeviceVector.from_host(v, ctx=ctx, capacity=capacity)


class DeviceConstraint:
    """A class-form constraint ``1/2 X'MX + v.X + c`` (``solvers.py:22-36``) whose operators are
    already resident in HBM: ``M`` a :class:`DeviceMatrix` or None, ``v`` a :class:`DeviceVector`
    or None.  ``solvers.cgmres`` takes it wherever the reference takes a constraint class."""

    def __init__(self, M, v, c):
        self.M, self.v, self.c = M, v, c


def device_constraints(conlist, ctx=None):
    """Upload the operators of reference-form class constraints once (``M`` dropped when it is
    all zeros, ``v`` when it is all zeros, as ``solvers.cgmres`` does per call)."""
    ctx = ctx or get_context()
    out = []
    for con in conlist:
        M = getattr(con, "M", None)
        if M is not None and not isinstance(M, DeviceMatrix):
            Ms = M if sps.issparse(M) else sps.csr_matrix(M)
            M = None if Ms.nnz == 0 or not np.any(Ms.data) else device_matrix(Ms, ctx=ctx)
        v = getattr(con, "v", None)
        if v is not None and not isinstance(v, DeviceVector):
            va = np.asarray(v, dtype=np.float64).reshape(-1)
            v = DeviceVector.from_host(va, ctx=ctx) if np.any(va) else None
        out.append(DeviceConstraint(M, v, float(np.asarray(getattr(con, "c", 0.0)))))
    return out
