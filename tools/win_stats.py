"""Column spans of the SpMV's row blocks: per natural 2,048-nnz row block of the
swe operator (the K1 table), the distinct 64-column chunks its nonzeros touch (the window K1w would
load), as a histogram, against the block's matrix bytes.  CPU only.

    python tools/win_stats.py [M]      (289: config C3, 913: C5)
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from structurepreservingiterativesolvers_amd.swe import assembly  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 289
A = assembly.linforms(M=M)[0]["A"]
rp, ci, n = A.indptr, A.indices, A.shape[0]
blocks, r = [0], 0
while r < n:  # rows never split, <= 2048 nnz per block (a longer row alone)
    r0 = r
    while r < n and rp[r + 1] - rp[r0] <= 2048:
        r += 1
    if r == r0:
        r += 1
    blocks.append(r)
ch = np.array([len(np.unique(ci[rp[blocks[b]]:rp[blocks[b + 1]]] >> 6)) for b in range(len(blocks) - 1)])
nz = np.diff(rp[blocks])
print(f"swe M={M}: N={n:,} nnz={A.nnz:,} blocks={len(ch):,} nnz/block {nz.mean():.0f}")
print(f"64-column chunks per block: mean {ch.mean():.1f} median {np.median(ch):.0f} max {ch.max()}")
print(f"window bytes per block ((x, z) pairs) {ch.mean() * 64 * 16 / 1024:.1f} KB vs matrix bytes {nz.mean() * 12 / 1024:.1f} KB")
edges = [0, 8, 12, 16, 20, 24, 28, 32, 40, 64, 10 ** 9]
h, _ = np.histogram(ch, bins=edges)
for lo, hi, c in zip(edges[:-1], edges[1:], h):
    print(f"  chunks [{lo:>3}, {hi if hi < 10 ** 9 else 'inf':>3}): {c:7d} blocks ({100.0 * c / len(ch):5.1f}%)")
