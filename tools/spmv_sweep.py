"""GPU: the solver's SpMV launches on a swe matrix (default C5, M = 913) under every SpMV kernel
family / column width (SPIS_OPT_SPMV_PIPE, SPIS_OPT_COL16), timed standalone by spis_spmv_bench
warm (back to back) and cold (behind a 1 GiB cache-evicting read):

    python tools/spmv_sweep.py [M] [modes...]

One line per configuration: kind (arnoldi / dual), us and algorithmic GB/s warm and cold."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from structurepreservingiterativesolvers_amd import _lib  # noqa: E402
from structurepreservingiterativesolvers_amd.device import get_context, set_option  # noqa: E402
from structurepreservingiterativesolvers_amd.swe import assembly  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 913
modes = sys.argv[2:] or ["xcd", "stride", "xcd_natural"]
dic, _ = assembly.linforms(M=M)
A = dic["A"]
n, nnz = A.shape[0], A.nnz
ctx = get_context(0)
print(f"M={M} N={n:,} nnz={nnz:,}", flush=True)
keys = [int(k) for k in os.environ.get("SPMV_SWEEP_KEYS", "1").split(",")]  # SPIS_OPT_SLAB_KEY values
configs = [(m, c16, key) for m in modes for c16 in (0, 2) for key in keys]
for mode, c16, key in configs:
    set_option("slab_key", key)
    set_option("spmv_pipe", mode)
    set_option("col16", {0: False, 2: True}[c16])
    from structurepreservingiterativesolvers_amd.device import DeviceMatrix

    Ad = DeviceMatrix(ctx, A)  # a fresh upload: the table / copies follow the options
    cb = 2 if c16 else 4
    for kind, name in ((0, "arnoldi"), (1, "dual")):
        byt = (8 + cb) * nnz + 4 * (n + 1) + (16 if kind == 0 else 32) * n
        res = []
        for cold in (0, 1):
            v = C.c_double()
            _lib.check(ctx.L.spis_spmv_bench(ctx.handle, Ad.handle, kind, cold, 20, C.byref(v)), "bench")
            res.append(v.value)
        print(f"{mode:12s} key={key} col16={c16} {name:8s} warm {res[0]:8.1f} us {byt / res[0] / 1e3:7.0f} GB/s | "
              f"cold {res[1]:8.1f} us {byt / res[1] / 1e3:7.0f} GB/s ({byt / res[1] / 1e3 / 8000:.3f})", flush=True)
    del Ad
set_option("spmv_pipe", "auto")
set_option("col16", "auto")
set_option("slab_key", True)
