"""A/B (GPU): the C3 / C5 system solved in its natural field-major numbering and in the
field-interleaved numbering (rows and columns of A and L symmetrically permuted; b, omega
permuted; each row's entries kept in their order), to measure what a bandwidth-reducing
permutation at upload would buy the SpMV gathers before building it into the library.

    python tools/perm_ab.py [M=289] [solves=20]
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sps

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from structurepreservingiterativesolvers_amd import _lib, solvers  # noqa: E402
from structurepreservingiterativesolvers_amd.device import (DeviceVector, device_constraints, device_matrix,  # noqa: E402
                                                            get_context)
from structurepreservingiterativesolvers_amd.swe import LinearSolver as ls  # noqa: E402
from structurepreservingiterativesolvers_amd.swe import assembly  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 289
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dic, _ = assembly.linforms(M=M)
A, L, b, om = dic["A"].tocsr(), dic["L"].tocsr(), dic["b"], dic["omega"]
n = A.shape[0]
sizes = [6 * M * M, 4 * M * M, 2 * M * M]
key = np.concatenate([(np.arange(s) + 0.5) / s for s in sizes])
P = np.argsort(key, kind="stable")
iperm = np.empty_like(P)
iperm[P] = np.arange(n)


def perm_csr(B):
    R = B[P].tocsr()  # rows in the new order, each row's entries in stored order
    return sps.csr_matrix((R.data, iperm[R.indices].astype(np.int32), R.indptr.astype(np.int32)), shape=B.shape)


ctx = get_context(0)
out = {}
for name, (AA, LL, bb, oo) in {"natural": (A, L, b, om),
                                "interleaved": (perm_csr(A), perm_csr(L), b[P].copy(), om[P].copy())}.items():
    d2 = dict(dic, A=AA, L=LL, b=bb, omega=oo)
    x0 = np.zeros(n)
    Ad = device_matrix(AA, ctx=ctx)
    bd = DeviceVector.from_host(bb, ctx=ctx)
    x0d = DeviceVector.from_host(x0, ctx=ctx)
    cons = device_constraints(ls.constraints(d2, x0), ctx=ctx)
    for _ in range(3):
        xs, dd = solvers.cgmres(Ad, bd, x0d, 30, tol=1e-19, conlist=cons)
    ctx.synchronize()
    _lib.check(ctx.L.spis_profile_enable(ctx.handle, 1), "prof")
    t0 = time.perf_counter()
    it = 0
    for _ in range(reps):
        xs, dd = solvers.cgmres(Ad, bd, x0d, 30, tol=1e-19, conlist=cons)
        it += dd["steps"]
    ctx.synchronize()
    el = time.perf_counter() - t0
    ms, cnt = _lib.profile_read(ctx.L, ctx.handle)
    _lib.check(ctx.L.spis_profile_enable(ctx.handle, 0), "prof")
    us = {}
    for cold in (0, 1):
        v = C.c_double()
        _lib.check(ctx.L.spis_spmv_bench(ctx.handle, Ad.handle, 1, cold, 20, C.byref(v)), "bench")
        us[cold] = v.value
    x = np.asarray(xs.numpy())
    if name == "interleaved":
        xn = np.empty(n)
        xn[P] = x
        x = xn
    out[name] = {"it_s": it / el, "dual_us": 1e3 * ms[_lib.PROF_SPMV_DUAL] / max(cnt[_lib.PROF_SPMV_DUAL], 1),
                 "mgs_us": 1e3 * ms[_lib.PROF_MGS] / max(cnt[_lib.PROF_MGS], 1),
                 "dual_standalone_warm_us": us[0], "dual_cold_us": us[1], "res_last": dd["res"][-1],
                 "x_norm": float(np.linalg.norm(x))}
    print(name, json.dumps(out[name]), flush=True)
xa = None
print(json.dumps({"M": M, "n": n, "nnz": A.nnz, **out}))
