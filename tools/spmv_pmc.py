"""GPU, under `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` (one pass each): the solver's
Arnoldi SpMV and fused dual SpMV launches on a bench configuration's matrix, standalone with the
solver's default kernel choice (spis_spmv_bench), so that the per-launch HBM traffic of both
SpMVs is measured:

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d DIR -o run -- python tools/spmv_pmc.py [CFG] [nt] [cold] [key]

CFG: c5 (default: swe M = 913, 1.25 GB of 16-bit-column matrix stream, where the matrix never
stays resident), c2 or c4 (lkdv / lkdvRK: the matrix fits the Infinity Cache, as in the solver),
or a bare number = swe M.  cold = 1 (default for c5): each launch behind the 1 GiB evicting read;
0: back to back, as the solver runs them.  Prints progress (the GPU box kills a command that
stays silent for 3 minutes)."""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from structurepreservingiterativesolvers_amd import _lib  # noqa: E402
from structurepreservingiterativesolvers_amd.device import device_matrix, get_context  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
nt = int(sys.argv[2]) if len(sys.argv) > 2 else 0  # SPIS_OPT_SPMV_NT for an A/B pass
if cfg.isdigit():
    wl = bench.build_workload(argparse.Namespace(config="c5", M=int(cfg), cycles=1))
    cfg = "c5"
else:
    wl = bench.build_workload(argparse.Namespace(config=cfg, M=None, cycles=1))
cold = int(sys.argv[3]) if len(sys.argv) > 3 else (1 if cfg == "c5" else 0)
key = int(sys.argv[4]) if len(sys.argv) > 4 else 1  # SPIS_OPT_SLAB_KEY at upload
print(f"assembled {cfg}: N={wl['A'].shape[0]:,} nnz={wl['A'].nnz:,}", flush=True)
ctx = get_context(0)
_lib.check(ctx.L.spis_set_option(ctx.handle, _lib.OPT_SPMV_NT, nt), "spis_set_option")
_lib.check(ctx.L.spis_set_option(ctx.handle, _lib.OPT_SLAB_KEY, key), "spis_set_option")
Ad = device_matrix(wl["A"], ctx=ctx)
for kind, name in ((0, "arnoldi"), (1, "dual")):
    v = C.c_double()
    _lib.check(ctx.L.spis_spmv_bench(ctx.handle, Ad.handle, kind, cold, 5, C.byref(v)), "spis_spmv_bench")
    print(f"{name}: {v.value:.1f} us ({'cold' if cold else 'warm'}, under the profiler)", flush=True)
