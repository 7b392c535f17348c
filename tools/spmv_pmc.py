"""GPU, under `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` (one pass each): the solver's
Arnoldi SpMV and fused dual SpMV launches on the C5 swe matrix (M = 913, 1.25 GB of 16-bit-column
matrix stream), standalone behind the 1 GiB cache-evicting read (spis_spmv_bench, cold), with the
solver's default kernel choice, so the per-launch HBM traffic of both SpMVs is measured at the
size where the matrix never stays resident:

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d DIR -o run -- python tools/spmv_pmc.py [M] [nt]

Prints progress (the GPU box kills a command that stays silent for 3 minutes)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from structurepreservingiterativesolvers_amd import _lib  # noqa: E402
from structurepreservingiterativesolvers_amd.device import device_matrix, get_context  # noqa: E402
from structurepreservingiterativesolvers_amd.swe import assembly  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 913
nt = int(sys.argv[2]) if len(sys.argv) > 2 else 0  # SPIS_OPT_SPMV_NT for an A/B pass
dic, _ = assembly.linforms(M=M)
print(f"assembled M={M}", flush=True)
ctx = get_context(0)
_lib.check(ctx.L.spis_set_option(ctx.handle, _lib.OPT_SPMV_NT, nt), "spis_set_option")
Ad = device_matrix(dic["A"], ctx=ctx)
for kind, name in ((0, "arnoldi"), (1, "dual")):
    v = C.c_double()
    _lib.check(ctx.L.spis_spmv_bench(ctx.handle, Ad.handle, kind, 1, 5, C.byref(v)), "spis_spmv_bench")
    print(f"{name}: {v.value:.1f} us (cold, under the profiler)", flush=True)
