"""CPU: how often the SpMV's gathered x lines are re-fetched under each block order of the swe
operator (the slab order with and without the slab key, csrc/slab_order.h via liblsq_host.so).

    python tools/slab_locality.py [M] [rows_per_block]

Each XCD walks a contiguous eighth of the block table round-robin (about 100 blocks at a time),
so a 128-B line of x is re-fetched when its previous use in the same eighth lies more than D
blocks back (D ~ an XCD's 4 MB L2 over the bytes one block moves through it).  Printed per
order: lines fetched / distinct lines, for several D."""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from structurepreservingiterativesolvers_amd.swe import assembly  # noqa: E402

PI = C.POINTER(C.c_int32)


def blocks(rp, cap=2048, rows=256):
    """Row blocks of <= cap nonzeros and <= rows rows (the solver's table, long rows aside)."""
    out = [0]
    n = len(rp) - 1
    r = 0
    while r < n:
        r1 = min(n, r + rows)
        r1 = max(r + 1, int(np.searchsorted(rp, rp[r] + cap, side="right")) - 1) if rp[r1] - rp[r] > cap else r1
        out.append(r1)
        r = r1
    return np.asarray(out, dtype=np.int32)


def order(L, A, blk, keyed):
    rp = np.ascontiguousarray(A.indptr, dtype=np.int32)
    ci = np.ascontiguousarray(A.indices, dtype=np.int32)
    out = np.zeros(4 * (len(blk) - 1), dtype=np.int32)
    ok = L.slab_order_blocks_keyed(A.shape[0], rp.ctypes.data_as(PI), ci.ctypes.data_as(PI), blk.ctypes.data_as(PI),
                                   len(blk), out.ctypes.data_as(PI), int(keyed))
    return out.reshape(-1, 4)[:, [0, 2]] if ok else np.stack([blk[:-1], blk[1:]], axis=1)


def refetch(A, spans, dists):
    rp, ci = A.indptr, A.indices
    nb = len(spans)
    fetched = np.zeros(len(dists))
    distinct = 0
    for g in range(8):
        sel = spans[nb * g // 8: nb * (g + 1) // 8]
        pos, lines = [], []
        for p, (r0, r1) in enumerate(sel):
            ln = np.unique(ci[rp[r0]:rp[r1]] // 16)
            lines.append(ln)
            pos.append(np.full(ln.size, p, dtype=np.int64))
        pos, lines = np.concatenate(pos), np.concatenate(lines)
        o = np.lexsort((pos, lines))
        pos, lines = pos[o], lines[o]
        first = np.ones(lines.size, dtype=bool)
        first[1:] = lines[1:] != lines[:-1]
        gap = np.diff(pos, prepend=0)
        distinct += int(first.sum())
        for i, d in enumerate(dists):
            fetched[i] += first.sum() + ((~first) & (gap > d)).sum()
    return fetched, distinct


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 913
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    L = C.CDLL(os.path.join(ROOT, "structurepreservingiterativesolvers_amd", "liblsq_host.so"))
    L.slab_order_blocks_keyed.argtypes = [C.c_int64, PI, PI, PI, C.c_int64, PI, C.c_int32]
    L.slab_order_blocks_keyed.restype = C.c_int
    t = time.time()
    A = assembly.linforms(M=M)[0]["A"].tocsr()
    blk = blocks(A.indptr, rows=rows)
    print(f"M={M} N={A.shape[0]:,} nnz={A.nnz:,} blocks={len(blk) - 1:,} ({time.time() - t:.0f} s)", flush=True)
    dists = [48, 96, 192, 384]
    nat = np.stack([blk[:-1], blk[1:]], axis=1)
    total_lines = (A.shape[1] + 15) // 16
    for name, spans in (("natural", nat), ("slab", order(L, A, blk, False)), ("slab+key", order(L, A, blk, True))):
        f, d = refetch(A, spans, dists)
        print(f"{name:9s} distinct/total {d / total_lines:5.2f} | fetched/total " +
              " ".join(f"D={dd}: {ff / total_lines:5.2f}" for dd, ff in zip(dists, f)), flush=True)


if __name__ == "__main__":
    main()
