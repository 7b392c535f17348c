"""Single-thread x0 scan + b copy (C3 size) in a bare process after a chosen import set, to find
what makes the drop-in's host copies slow in the bench process (tools/r06_h2d_probe.py)."""
import ctypes as C
import sys
import time

mode = sys.argv[1]
if mode in ("torch", "torch_bench"):
    import torch  # noqa: F401
if mode in ("bench", "torch_bench"):
    sys.path.insert(0, ".")
    import bench  # noqa: F401
if mode == "pkg":
    sys.path.insert(0, ".")
    import structurepreservingiterativesolvers_amd  # noqa: F401
import numpy as np  # noqa: E402

sys.path.insert(0, ".")
from structurepreservingiterativesolvers_amd import _lib  # noqa: E402

L = _lib.load_library()
n = 196608
x0 = np.zeros(n)
b = np.random.default_rng(0).random(n)
d = np.empty(n)
r = C.c_int32()
for rep in range(3):
    t = time.perf_counter()
    for _ in range(100):
        L.spis_host_nonzero(C.c_void_p(x0.ctypes.data), C.c_int64(n), 1, 1, C.byref(r))
        L.spis_host_copy(C.c_void_p(d.ctypes.data), C.c_void_p(b.ctypes.data), C.c_int64(b.nbytes), 1)
    print(f"{mode}: scan+copy (1 thread) {(time.perf_counter() - t) / 100 * 1e6:.1f} us", flush=True)
