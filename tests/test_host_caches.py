"""Host-side upload / zero-test caches (device.py): keyed on identity + buffer addresses, evicted
with the object, and re-verified against a digest of the full contents on every use
(spis_host_hash).  CPU only: no upload happens here (the hash runs in libspis.so without a device)."""
import gc

import numpy as np
import pytest
import scipy.sparse as sps

from structurepreservingiterativesolvers_amd import _lib, device


def _mat(seed, zero=False, n=500):
    rng = np.random.default_rng(seed)
    A = sps.random(n, n, density=0.02, random_state=rng, format="csr") + sps.identity(n, format="csr")
    A = sps.csr_matrix(A)
    return 0 * A if zero else A


@pytest.fixture(autouse=True)
def _need_lib():
    try:
        _lib.load_library()
    except _lib.SpisUnavailable as e:  # pragma: no cover - the build is part of the suite's set-up
        pytest.skip(str(e))


def test_zero_cache_evicted_with_object():
    """The reference wrappers' mass is 0*A (A's pattern, zero values).  A later, different matrix
    that happens to reuse the freed object's id must not inherit its 'zero' verdict."""
    M = _mat(0, zero=True)
    assert M.nnz > 0 and device.is_zero_matrix(M)
    key = device._matrix_key(M)
    assert key in device._ZERO_CACHE
    del M
    gc.collect()
    assert key not in device._ZERO_CACHE
    for seed in range(20):  # same shape and nnz: ids are reused by CPython
        N = _mat(seed)
        assert not device.is_zero_matrix(N)
        del N


@pytest.mark.parametrize("where", [0, 1, 4097, -1])
def test_zero_cache_sees_any_in_place_change(where):
    """Every entry is covered, not a sample: entries 1 and 4097 fell between round 3's 256 sampled
    positions at this size."""
    M = _mat(1, zero=True)
    assert device.is_zero_matrix(M)
    M.data[where] = 1.0
    assert not device.is_zero_matrix(M)
    M.data[where] = 0.0
    assert device.is_zero_matrix(M)


def test_deferred_check_reports_a_stale_entry():
    """With a check list (solvers._run), a large cached entry is verified on the verifier thread;
    an in-place edit makes the pending check fail and drops the entry."""
    M = _mat(3, zero=True, n=40_000)
    assert device._nbytes(M) >= device._ASYNC_MIN_BYTES
    assert device.is_zero_matrix(M)
    checks = []
    assert device.is_zero_matrix(M, checks) and len(checks) == 1
    assert checks[0].ok()
    M.data[M.nnz // 2 + 1] = 2.0
    checks = []
    assert device.is_zero_matrix(M, checks)  # the stale cached verdict, checked beside the work
    assert not checks[0].ok()
    assert device._matrix_key(M) not in device._ZERO_CACHE
    assert not device.is_zero_matrix(M)


def test_invalidate_forgets_entries():
    M = _mat(2, zero=True)
    assert device.is_zero_matrix(M)
    device.invalidate(M)
    assert device._matrix_key(M) not in device._ZERO_CACHE
    assert device.is_zero_matrix(M)
    device.invalidate()
    assert not device._ZERO_CACHE


def test_content_digest_sees_every_entry():
    for n in (1, 7, 5000, 100_000):
        A = sps.csr_matrix(sps.diags([np.arange(1.0, n + 1)], [0]) + sps.eye(n, k=1))
        f = device.content_digest(A)
        assert device.content_digest(A.copy()) == f
        for i in {0, A.nnz // 3, A.nnz - 1}:
            B = A.copy()
            B.data[i] = np.nextafter(B.data[i], np.inf)  # one ulp of one entry
            assert device.content_digest(B) != f
        B = A.copy()
        B.indices[-1] = (B.indices[-1] + 1) % n if n > 1 else 0
        if n > 1:
            assert device.content_digest(B) != f


@pytest.mark.parametrize("n", [5, 6, 7, 1001, 1002, 1003])
def test_content_digest_sees_swapped_tail_entries(n):
    """Swaps among the last (bytes mod 32) bytes: the tail is hashed by position, so swapping the
    last two values, or indices[-1] with indices[-3] (8 bytes apart), changes the digest."""
    rng = np.random.default_rng(n)
    A = sps.csr_matrix(sps.random(n, n, density=0.3, random_state=rng) + sps.eye(n))
    f = device.content_digest(A)
    B = A.copy()
    B.data[[-1, -2]] = B.data[[-2, -1]]
    assert not np.array_equal(B.data, A.data) and device.content_digest(B) != f
    C = A.copy()
    C.indices[[-1, -3]] = C.indices[[-3, -1]]
    if not np.array_equal(C.indices, A.indices):
        assert device.content_digest(C) != f
    for k in range(1, 32):  # one tail byte at every tail position, and a same-XOR pair 8 apart
        raw = np.frombuffer(A.data.tobytes(), np.uint8).copy()
        if k + 8 > raw.size:
            break
        raw[-k] ^= 0x5A
        raw[-k - 8] ^= 0x5A
        D = A.copy()
        D.data = np.frombuffer(raw.tobytes(), np.float64).copy()
        assert device.content_digest(D) != f


def test_host_hash_independent_of_threads():
    import ctypes as C

    L = _lib.load_library()
    a = np.random.default_rng(0).random(3 << 20)  # 24 MiB: several pieces per thread
    outs = set()
    for t in (1, 2, 3, 8):
        h = C.c_uint64()
        _lib.check(L.spis_host_hash(C.c_void_p(a.ctypes.data), a.nbytes, t, C.byref(h)), "spis_host_hash")
        outs.add(h.value)
    assert len(outs) == 1
    h2 = C.c_uint64()
    a[12345] = np.nextafter(a[12345], 2.0)
    _lib.check(L.spis_host_hash(C.c_void_p(a.ctypes.data), a.nbytes, 4, C.byref(h2)), "spis_host_hash")
    assert h2.value not in outs


def test_host_nonzero_matches_numpy_truthiness():
    """spis_host_nonzero is np.any on fp64 entries: -0.0 is zero, NaN and subnormals are not; a
    lone nonzero anywhere (head, a pooled piece, the ragged tail) is found."""
    n = (3 << 20) + 77  # head + several 1 MiB pieces + a tail
    z = np.zeros(n)
    assert device.host_nonzero(z) is False
    z[::3] = -0.0
    assert device.host_nonzero(z) is False and bool(np.any(z)) is False
    for pos in (0, 4095, 4096, n // 2, n - 1):
        for val in (1.0, np.nan, 5e-324, -np.inf):
            w = np.zeros(n)
            w[pos] = val
            assert device.host_nonzero(w) is True, (pos, val)
    assert device.host_nonzero(np.zeros(0)) is False
    assert device.host_nonzero(np.zeros(10)[::2]) is False  # non-contiguous: numpy's own any
    assert device.host_nonzero(np.arange(10.0)[::2]) is True


def test_host_hash_concurrent_callers():
    """Two threads hashing at once (the verifier thread and an inline check) both get the
    digest a lone caller gets: one of them runs on the pool, the other on its own thread."""
    import threading

    rng = np.random.default_rng(3)
    arrs = [rng.random(5 << 20) for _ in range(2)]
    want = [device.vector_digest(a) for a in arrs]
    got = [[], []]

    def worker(i):
        for _ in range(5):
            got[i].append(device.vector_digest(arrs[i]))

    th = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert got[0] == [want[0]] * 5 and got[1] == [want[1]] * 5


def test_vector_cache_keyed_on_owner():
    """A constraint vector passed as a fresh view each call (np.transpose(omega),
    swe/LinearSolver.py:28) keys on its owner: the entry lives as long as omega, not the view."""
    key_of = lambda a: (id(device._root(a)), device._root(a).ctypes.data, a.ctypes.data, a.size)  # noqa: E731
    omega = np.random.default_rng(1).random(1000)
    v1, v2 = np.transpose(omega), np.transpose(omega)
    assert v1 is not v2 and key_of(v1) == key_of(v2) == (id(omega), omega.ctypes.data, omega.ctypes.data, 1000)


def test_host_nonzero_bitwise_counts_negative_zero():
    """The x0 test is bitwise: an x0 of -0.0 entries is uploaded as given (its sign reaches
    x_j = Z y + x0), only +0.0 entries take the shared zero vector."""
    n = (2 << 20) + 3
    z = np.zeros(n)
    assert device.host_nonzero(z, bitwise=True) is False
    for pos in (0, 5000, n - 1):
        w = np.zeros(n)
        w[pos] = -0.0
        assert device.host_nonzero(w, bitwise=True) is True
        assert device.host_nonzero(w) is False


def test_host_copy_exact():
    """spis_host_copy (the staging copy of b): every length, aligned (streaming stores) and not."""
    import ctypes as C

    from structurepreservingiterativesolvers_amd import _lib

    L = _lib.load_library()
    for n in (0, 1, 7, 100, 1 << 15, (1 << 15) + 3, 1000003):
        a = np.random.default_rng(n).random(n)
        d = np.zeros(n)
        assert L.spis_host_copy(C.c_void_p(d.ctypes.data), C.c_void_p(a.ctypes.data), a.nbytes, 8) == 0
        assert np.array_equal(a, d), n
        s = np.frombuffer(a.tobytes(), dtype=np.uint8)
        t = np.zeros(s.size + 1, np.uint8)
        assert L.spis_host_copy(C.c_void_p(t.ctypes.data + 1), C.c_void_p(s.ctypes.data), s.size, 8) == 0
        assert np.array_equal(t[1:], s), n


def test_x0_zero_verdict_cached_and_rechecked(monkeypatch):
    """device.host_x0_zero: a first sight scans once (inline); a repeat takes the cached verdict and,
    from 4 MiB, queues the re-check on the verifier thread; an in-place edit fails that check, which
    evicts the entry, so the next call scans inline again."""
    scans = []
    real = device.host_nonzero
    monkeypatch.setattr(device, "host_nonzero", lambda v, bitwise=False: scans.append(v.size) or real(v, bitwise))
    n = (device._ASYNC_MIN_BYTES // 8) + 5
    x0 = np.zeros(n)
    assert device.host_x0_zero(x0) is True and len(scans) == 1
    checks = []
    assert device.host_x0_zero(x0, checks) is True and len(checks) == 1
    assert checks[0].ok() is True and len(scans) == 2
    x0[n - 1] = 1.0
    checks = []
    assert device.host_x0_zero(x0, checks) is True  # the speculative verdict ...
    assert checks[0].ok() is False  # ... which the re-check refutes (the caller re-runs)
    assert device.host_x0_zero(x0) is False  # evicted: scanned inline
    small = np.zeros(100)
    assert device.host_x0_zero(small, []) is True
    small[99] = -0.0
    assert device.host_x0_zero(small, []) is False  # below 4 MiB: re-checked inline, bitwise
    device.invalidate()


@pytest.mark.gpu
def test_pinned_buffers_recycled_and_capped():
    """Returned iterates live in page-locked buffers (device.pinned_empty): a dropped array's buffer
    is reused, every view keeps it alive, and past the cap per length downloads fall back to
    ordinary arrays (None here)."""
    n = 1000 + 7
    a = device.pinned_empty(n)
    assert a is not None and a.shape == (n,) and a.dtype == np.float64
    a[:] = 3.0
    addr = a.ctypes.data
    view = a[10:20]
    del a
    gc.collect()
    assert (view == 3.0).all()  # the view keeps the buffer
    del view
    gc.collect()
    b = device.pinned_empty(n)
    assert b.ctypes.data == addr  # recycled
    held = [b] + [device.pinned_empty(n) for _ in range(device._PINNED_MAX - 1)]
    assert all(h is not None for h in held)
    assert device.pinned_empty(n) is None  # capped
    del held, b
    gc.collect()
    assert device.pinned_empty(n) is not None



def test_staged_upload_slots(monkeypatch):
    """device._stage: a call's b (and nonzero x0) go through two page-locked staging buffers per
    size, used in turn; a slot is rewritten without a context synchronize only when a solve has
    returned since its last upload (that solve's stream ran the upload first).  The library is
    stubbed (no HIP runtime here)."""
    calls = []

    class FakeLib:
        def __init__(self):
            self.next_ptr = 1 << 20

        def spis_host_alloc(self, nbytes, out):
            out._obj.value = self.next_ptr
            self.next_ptr += 1 << 24
            calls.append(("alloc", nbytes))
            return _lib.OK

        def spis_host_free(self, p):
            calls.append(("free", p.value))
            return _lib.OK

        def spis_host_copy(self, dst, src, nbytes, threads):
            calls.append(("copy", dst.value))
            return _lib.OK

        def spis_memcpy_h2d_async(self, h, dst, src, nbytes):
            calls.append(("h2d", src.value))
            return _lib.OK

    class FakeCtx:
        def __init__(self):
            self.L = FakeLib()
            self.token = -12345
            self.handle = None
            self.solves = 0

        def synchronize(self):
            calls.append(("sync",))

    class Dev:
        ptr = 777

    fake = FakeCtx()
    monkeypatch.setattr(_lib, "load_library", lambda *a: fake.L)
    monkeypatch.setattr(device, "_STAGING", {})
    a = np.ones(1 << 18)  # 2 MiB
    assert device._stage(fake, Dev(), a) and device._stage(fake, Dev(), a)  # b, x0 of one call
    s0, s1 = [c[1] for c in calls if c[0] == "copy"]
    assert s0 != s1 and ("sync",) not in calls and [c[0] for c in calls].count("alloc") == 2
    calls.clear()
    assert device._stage(fake, Dev(), a)  # no solve since slot 0's upload: wait for it
    assert calls[0] == ("sync",) and calls[1] == ("copy", s0)
    calls.clear()
    fake.solves += 1  # a solve returned
    assert device._stage(fake, Dev(), a) and calls == [("copy", s1), ("h2d", s1)]
