"""Slab order of the SpMV row blocks (csrc/slab_order.h via the host-only liblsq_host.so), on CPU.

The XCD-local SpMV walk (SPIS_OPT_SPMV_PIPE 2, the default at C3) gives each XCD a contiguous
eighth of the block table.  The upload reorders the table so that an eighth is a spatial slab
across the DoF groups the FE numbering puts one after another; rows are untouched.  Checked here:
the table is a permutation of the blocks with consistent nz offsets, the share of 128-B lines of
the gathered vector that several eighths touch drops on the swe matrix (M=30), and a banded
matrix (already slab-like) keeps its natural order.  The 16-bit column copy of the same blocks
(csrc/col16.h) decodes to the original columns exactly, and is refused for a block that spans
more than four ranges of 2^14 columns."""
import ctypes as C
import os

import numpy as np
import pytest
import scipy.sparse as sps

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "structurepreservingiterativesolvers_amd", "liblsq_host.so")
PI = C.POINTER(C.c_int32)


@pytest.fixture(scope="module")
def host():
    if not os.path.exists(LIB):
        pytest.skip("liblsq_host.so not built (make)")
    L = C.CDLL(LIB)
    L.slab_order_blocks.argtypes = [C.c_int64, PI, PI, PI, C.c_int64, PI]
    L.slab_order_blocks.restype = C.c_int
    return L


def _blocks(A, rows=256):
    n = A.shape[0]
    return np.ascontiguousarray(np.append(np.arange(0, n, rows), n), dtype=np.int32)


def _order(host, A, blk):
    rp = np.ascontiguousarray(A.indptr, dtype=np.int32)
    ci = np.ascontiguousarray(A.indices, dtype=np.int32)
    out = np.zeros(4 * (len(blk) - 1), dtype=np.int32)
    ok = host.slab_order_blocks(A.shape[0], rp.ctypes.data_as(PI), ci.ctypes.data_as(PI), blk.ctypes.data_as(PI),
                                len(blk), out.ctypes.data_as(PI))
    return ok, out.reshape(-1, 4)


def _lines_per_eighth(A, spans):
    """Sum over eighths of the table of the 16-entry lines of x its rows gather / total lines."""
    rp, ci = A.indptr, A.indices
    nb = len(spans)
    tot = 0
    for g in range(8):
        sel = spans[nb * g // 8: nb * (g + 1) // 8]
        cols = np.concatenate([ci[rp[r0]:rp[r1]] for r0, r1 in sel])
        tot += np.unique(cols // 16).size
    return tot / ((A.shape[1] + 15) // 16)


def test_swe_slab_order(host):
    from structurepreservingiterativesolvers_amd.swe import assembly as sa

    dic, _ = sa.linforms(M=30)
    A = dic["A"].tocsr()
    blk = _blocks(A)
    ok, pairs = _order(host, A, blk)
    assert ok == 1
    # a permutation of the blocks, nz offsets from indptr
    natural = np.stack([blk[:-1], blk[1:]], axis=1)
    got = pairs[:, [0, 2]]
    assert sorted(map(tuple, got)) == sorted(map(tuple, natural))
    np.testing.assert_array_equal(pairs[:, 1], A.indptr[pairs[:, 0]])
    np.testing.assert_array_equal(pairs[:, 3], A.indptr[pairs[:, 2]])
    before = _lines_per_eighth(A, natural)
    after = _lines_per_eighth(A, got)
    assert before > 3.0 and after < 0.6 * before, (before, after)  # C3 (M=289): 3.0 -> 1.14


def _refetched_lines(A, spans, dist):
    """Lines of x fetched per eighth when a line whose previous use in that eighth lies more than
    dist blocks back is fetched again (an XCD's L2 over its round-robin walk), / total lines."""
    rp, ci = A.indptr, A.indices
    nb = len(spans)
    fetched = 0
    for g in range(8):
        sel = spans[nb * g // 8: nb * (g + 1) // 8]
        lines = [np.unique(ci[rp[r0]:rp[r1]] // 16) for r0, r1 in sel]
        pos = np.concatenate([np.full(ln.size, p) for p, ln in enumerate(lines)])
        lines = np.concatenate(lines)
        o = np.lexsort((pos, lines))
        pos, lines = pos[o], lines[o]
        first = np.ones(lines.size, dtype=bool)
        first[1:] = lines[1:] != lines[:-1]
        fetched += first.sum() + ((~first) & (np.diff(pos, prepend=0) > dist)).sum()
    return fetched / ((A.shape[1] + 15) // 16)


def test_swe_slab_key_walks_groups_side_by_side(host):
    """SPIS_OPT_SLAB_KEY: inside a slab the blocks follow their rows' position, so an x line's
    uses by the slab's edge, interior and rho blocks lie close together in the walk.  M = 240 with
    16-row blocks has C5's proportions (a slab ~6 times the reuse distance, which spans two mesh
    rows): group after group each line is fetched 1.53 times per eighth, side by side 1.05."""
    from structurepreservingiterativesolvers_amd.swe import assembly as sa

    A = sa.linforms(M=240)[0]["A"].tocsr()
    blk = _blocks(A, rows=16)
    host.slab_order_blocks_keyed.argtypes = [C.c_int64, PI, PI, PI, C.c_int64, PI, C.c_int32]
    host.slab_order_blocks_keyed.restype = C.c_int
    spans = {}
    for key in (0, 1):
        rp = np.ascontiguousarray(A.indptr, dtype=np.int32)
        ci = np.ascontiguousarray(A.indices, dtype=np.int32)
        out = np.zeros(4 * (len(blk) - 1), dtype=np.int32)
        assert host.slab_order_blocks_keyed(A.shape[0], rp.ctypes.data_as(PI), ci.ctypes.data_as(PI),
                                            blk.ctypes.data_as(PI), len(blk), out.ctypes.data_as(PI), key) == 1
        pairs = out.reshape(-1, 4)
        np.testing.assert_array_equal(pairs[:, 1], A.indptr[pairs[:, 0]])
        spans[key] = pairs[:, [0, 2]]
    natural = sorted(map(tuple, np.stack([blk[:-1], blk[1:]], axis=1)))
    assert sorted(map(tuple, spans[1])) == natural  # a permutation of the blocks
    grouped, keyed = _refetched_lines(A, spans[0], 360), _refetched_lines(A, spans[1], 360)
    assert keyed < 1.1 and grouped > 1.3 * keyed, (grouped, keyed)
    assert _lines_per_eighth(A, spans[1]) <= _lines_per_eighth(A, spans[0])


def test_banded_keeps_natural_order(host):
    n = 20000
    A = sps.diags([np.ones(n - 1), 2 * np.ones(n), np.ones(n - 1)], [-1, 0, 1], format="csr")
    ok, _ = _order(host, A, _blocks(A))
    assert ok == 0


def test_too_few_blocks(host):
    A = sps.random(1000, 1000, density=0.01, format="csr", random_state=1)
    ok, _ = _order(host, A, _blocks(A, rows=256))
    assert ok == 0


# ---- the 16-bit column copy (csrc/col16.h) ------------------------------------------------------
def _col16(host, A, blk):
    rp = np.ascontiguousarray(A.indptr, dtype=np.int32)
    ci = np.ascontiguousarray(A.indices, dtype=np.int32)
    c16 = np.zeros(max(A.nnz, 1), dtype=np.uint16)
    bases = np.zeros(4 * (len(blk) - 1), dtype=np.int32)
    host.col16_encode.argtypes = [PI, PI, PI, C.c_int64, C.POINTER(C.c_uint16), PI]
    host.col16_encode.restype = C.c_int
    ok = host.col16_encode(rp.ctypes.data_as(PI), ci.ctypes.data_as(PI), blk.ctypes.data_as(PI), len(blk),
                           c16.ctypes.data_as(C.POINTER(C.c_uint16)), bases.ctypes.data_as(PI))
    return ok, c16, bases.reshape(-1, 4)


def _decode(A, blk, c16, bases):
    out = np.empty(A.nnz, dtype=np.int64)
    for b in range(len(blk) - 1):
        e0, e1 = A.indptr[blk[b]], A.indptr[blk[b + 1]]
        v = c16[e0:e1].astype(np.int64)
        out[e0:e1] = bases[b][v >> 14] + (v & 0x3FFF)
    return out


def test_col16_round_trip_swe(host):
    """Every column of the swe operator decodes exactly from (2-bit base index, 14-bit offset)."""
    from structurepreservingiterativesolvers_amd.swe import assembly as sa

    A = sa.linforms(M=30)[0]["A"].tocsr()
    blk = _blocks(A, rows=200)
    ok, c16, bases = _col16(host, A, blk)
    assert ok == 1
    np.testing.assert_array_equal(_decode(A, blk, c16, bases), A.indices)


def test_col16_long_row_and_refusal(host):
    # one long row over 3 ranges decodes; a row over 5 distant ranges has no 16-bit copy
    n = 100000
    cols = np.array([0, 1, 20000, 20001, 70000, 99999])
    A = sps.csr_matrix((np.ones(6), (np.zeros(6, dtype=int), cols)), shape=(n, n))
    blk = np.array([0, 1, n], dtype=np.int32)
    ok, c16, bases = _col16(host, A, blk)
    assert ok == 1
    np.testing.assert_array_equal(_decode(A, blk, c16, bases), A.indices)
    cols = np.array([0, 20000, 40000, 60000, 80000])
    A = sps.csr_matrix((np.ones(5), (np.zeros(5, dtype=int), cols)), shape=(n, n))
    ok, _, _ = _col16(host, A, blk)
    assert ok == 0
