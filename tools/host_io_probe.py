"""GPU box: the host pieces of a drop-in C3 call, each timed alone (median of 50): the zero
scans, the digest, an 8 MB upload (pageable; registered + asynchronous), the download (pageable;
page-locked by DMA; page-locked by a copy kernel storing into mapped host memory).

    python tools/host_io_probe.py
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from structurepreservingiterativesolvers_amd import _lib, device  # noqa: E402
from structurepreservingiterativesolvers_amd.device import DeviceVector, get_context  # noqa: E402
from structurepreservingiterativesolvers_amd.swe import LinearSolver as ls  # noqa: E402
from structurepreservingiterativesolvers_amd.swe import assembly  # noqa: E402


def med(fn, reps=50):
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return 1e3 * float(np.median(ts))


ctx = get_context(0)
L = ctx.L
dic, _ = assembly.linforms(M=289)
n = dic["A"].shape[0]
b = dic["b"]
z = np.zeros(n)
out = {}
out["nonzero_zeros_ms"] = med(lambda: device.host_nonzero(z, bitwise=True))
out["digest_A_ms"] = med(lambda: device.content_digest(dic["A"]), 10)
d = DeviceVector(ctx, n)
out["h2d_pageable_ms"] = med(lambda: d.upload(b))
t = time.perf_counter()
_lib.check(L.spis_host_register(C.c_void_p(b.ctypes.data), b.nbytes), "register")
out["register_ms"] = 1e3 * (time.perf_counter() - t)
out["h2d_registered_ms"] = med(lambda: d.upload(b))


def h2d_async():
    _lib.check(L.spis_memcpy_h2d_async(ctx.handle, C.c_void_p(d.ptr), C.c_void_p(b.ctypes.data), b.nbytes), "a")


out["h2d_async_issue_ms"] = med(h2d_async)
ctx.synchronize()
out["h2d_async_issue_plus_sync_ms"] = med(lambda: (h2d_async(), ctx.synchronize()))
_lib.check(L.spis_host_unregister(C.c_void_p(b.ctypes.data)), "unregister")
out["d2h_pageable_ms"] = med(lambda: d.download())
pinned = device.pinned_empty(n)
PD = C.POINTER(C.c_double)
out["d2h_pinned_dma_ms"] = med(lambda: _lib.check(L.spis_memcpy_d2h(ctx.handle, pinned.ctypes.data_as(C.c_void_p),
                                                                    C.c_void_p(d.ptr), 8 * n), "d2h"))
out["d2h_pinned_kernel_ms"] = med(lambda: _lib.check(L.spis_copy_to_host(ctx.handle, pinned.ctypes.data_as(PD),
                                                                         C.c_void_p(d.ptr), n), "copy"))
ref = d.download()
out["kernel_copy_exact"] = bool(np.array_equal(pinned, ref))
x0 = np.zeros(n)
out["wrapper_constraints_ms"] = med(lambda: ls.constraints(dic, x0))
print(json.dumps(out, indent=1))
