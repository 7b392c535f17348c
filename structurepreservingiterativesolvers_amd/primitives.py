"""NumPy-in / NumPy-out access to the individual HIP kernels of the inner loop
(tests, diagnostics, and callers that want one operation on the device).

Each function mirrors one reference expression:
``spmv`` = ``A @ z`` (solvers.py:191), ``residual_norm`` = ``||A.dot(x) - b||``
(:290), ``dot`` = ``np.dot`` (:194), ``axpy`` = ``y - h*q`` (:195), ``nrm2`` =
``np.linalg.norm`` (:196), ``gemv`` = ``Z @ y + x0`` (:287), ``gram`` = the
``Z.T @ MZ`` family of constraint_container (:33-36)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .device import DeviceVector, device_matrix, get_context

_PD = C.POINTER(C.c_double)


def _vec(a, ctx, capacity=None):
    return DeviceVector.from_host(np.asarray(a, dtype=np.float64), ctx=ctx, capacity=capacity)


def spmv(A, x):
    ctx = get_context()
    Ad = device_matrix(A, ctx=ctx)
    xd = _vec(x, ctx, capacity=Ad.shape[1])
    yd = DeviceVector(ctx, Ad.shape[0])
    _lib.check(ctx.L.spis_spmv(ctx.handle, Ad.handle, C.c_void_p(xd.ptr), C.c_void_p(yd.ptr)), "spis_spmv")
    return yd.numpy()


def residual_norm(A, x, b):
    ctx = get_context()
    Ad = device_matrix(A, ctx=ctx)
    xd, bd = _vec(x, ctx, capacity=Ad.shape[1]), _vec(b, ctx)
    out = C.c_double()
    _lib.check(ctx.L.spis_residual_norm(ctx.handle, Ad.handle, C.c_void_p(xd.ptr), C.c_void_p(bd.ptr), C.byref(out)),
               "spis_residual_norm")
    return out.value


def dot(x, y):
    ctx = get_context()
    xd, yd = _vec(x, ctx), _vec(y, ctx)
    out = C.c_double()
    _lib.check(ctx.L.spis_dot(ctx.handle, len(xd), C.c_void_p(xd.ptr), C.c_void_p(yd.ptr), C.byref(out)), "spis_dot")
    return out.value


def nrm2(x):
    ctx = get_context()
    xd = _vec(x, ctx)
    out = C.c_double()
    _lib.check(ctx.L.spis_nrm2(ctx.handle, len(xd), C.c_void_p(xd.ptr), C.byref(out)), "spis_nrm2")
    return out.value


def axpy(h, q, y):
    """``y - h*q`` (numpy semantics: product rounded, then subtracted)."""
    ctx = get_context()
    qd, yd = _vec(q, ctx), _vec(y, ctx)
    _lib.check(ctx.L.spis_axpy(ctx.handle, len(qd), float(h), C.c_void_p(qd.ptr), C.c_void_p(yd.ptr)), "spis_axpy")
    return yd.numpy()


def gemv(Z, y, x0):
    """``Z.T @ y + x0`` for Z stored row-major (p, n) like the reference's ``z``."""
    ctx = get_context()
    Z = np.ascontiguousarray(Z, dtype=np.float64)
    p, n = Z.shape
    Zd = _vec(Z.reshape(-1), ctx)
    x0d = _vec(x0, ctx)
    xd = DeviceVector(ctx, n)
    yv = np.ascontiguousarray(y, dtype=np.float64)
    _lib.check(ctx.L.spis_gemv(ctx.handle, n, p, C.c_void_p(Zd.ptr), n, yv.ctypes.data_as(_PD), C.c_void_p(x0d.ptr),
                               C.c_void_p(xd.ptr)), "spis_gemv")
    return xd.numpy()


def gram(U, V):
    """``G[a, b] = U[a] . V[b]`` (tall-skinny Gram, deterministic reduction)."""
    ctx = get_context()
    Ud = [_vec(u, ctx) for u in U]
    Vd = [_vec(v, ctx) for v in V]
    n = len(Ud[0])
    up = (C.c_void_p * len(Ud))(*[u.ptr for u in Ud])
    vp = (C.c_void_p * len(Vd))(*[v.ptr for v in Vd])
    G = np.zeros((len(Ud), len(Vd)))
    _lib.check(ctx.L.spis_gram(ctx.handle, n, len(Ud), up, len(Vd), vp, G.ctypes.data_as(_PD)), "spis_gram")
    return G
