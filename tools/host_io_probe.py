"""GPU box: the host pieces of a drop-in C3 call, each timed alone (median of 50): the zero
scans, the digest, an 8 MB upload from pageable / registered memory, the download, and the
wrapper's own set-up.

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
dic, _ = assembly.linforms(M=289)
n = dic["A"].shape[0]
b = dic["b"]
z = np.zeros(n)
out = {}
out["nonzero_zeros_ms"] = med(lambda: device.host_nonzero(z))
out["nonzero_fresh_zeros_ms"] = med(lambda: device.host_nonzero(np.zeros(n)))
out["np_zeros_like_ms"] = med(lambda: np.zeros_like(b))
out["nonzero_b_ms"] = med(lambda: device.host_nonzero(b))
out["digest_omega_ms"] = med(lambda: device.vector_digest(dic["omega"]))
out["digest_A_ms"] = med(lambda: device.content_digest(dic["A"]), 10)
d = DeviceVector(ctx, n)
out["h2d_pageable_ms"] = med(lambda: d.upload(b))
out["d2h_pageable_ms"] = med(lambda: d.download())
hr = ctypes_lib = C.CDLL("libamdhip64.so")
hr.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
hr.hipHostUnregister.argtypes = [C.c_void_p]
t = time.perf_counter()
rc = hr.hipHostRegister(C.c_void_p(b.ctypes.data), b.nbytes, 0)
out["register_ms"] = 1e3 * (time.perf_counter() - t)
out["register_rc"] = rc
out["h2d_registered_ms"] = med(lambda: d.upload(b))
t = time.perf_counter()
hr.hipHostUnregister(C.c_void_p(b.ctypes.data))
out["unregister_ms"] = 1e3 * (time.perf_counter() - t)
x0 = np.zeros(n)
out["wrapper_constraints_ms"] = med(lambda: ls.constraints(dic, x0))
print(json.dumps(out, indent=1))
