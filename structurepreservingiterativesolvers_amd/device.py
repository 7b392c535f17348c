"""Device-side handles: context, HBM-resident CSR matrices and vectors.

The reference hands SciPy CSR matrices and NumPy vectors to ``solvers.cgmres``
on every call (e.g. ``swe/LinearSolver.py:46``) and never mutates them
(``solvers.py:167`` allocates).  This module keeps one HBM copy per matrix
object: uploads are cached on ``id(A)`` and the addresses of its three arrays
(``data``/``indices``/``indptr``), dropped when the SciPy object is garbage
collected, and every solver call re-verifies the cached copy against a digest of
the arrays' full contents (``spis_host_hash``), on a host thread beside the solve:
an in-place edit of any entry is detected and the solve is redone on the new
values (:func:`device_matrix`).
"""
from __future__ import annotations

import ctypes as C
import os
import queue
import threading
import weakref

import numpy as np
import scipy.sparse as sps

from . import _lib

_DOUBLE_P = C.POINTER(C.c_double)
_I32_P = C.POINTER(C.c_int32)


_CTX_TOKENS = iter(range(1, 1 << 62))


class Context:
    """One HIP device + stream (+ optional RCCL communicator)."""

    def __init__(self, device=0):
        self.L = _lib.lib()
        self.token = next(_CTX_TOKENS)  # never reused (an id() can be, after a Context is dropped)
        h = C.c_void_p()
        _lib.check(self.L.spis_context_create(int(device), C.byref(h)), "spis_context_create")
        self.handle = h
        self.device = int(device)
        self.nranks = 1
        self.rank = 0
        self.device_ilu = "auto"  # SuperLU preconditioners on the device (K8) where the plan predicts a win
        self.solves = 0  # spis_solve calls returned (device_vector's staging slots: see _stage)

    def synchronize(self):
        _lib.check(self.L.spis_context_synchronize(self.handle), "spis_context_synchronize")

    def close(self):
        """Destroy the context; device objects still alive become inert (their finalizers
        see the closed context and do nothing)."""
        if self.handle:
            for (tok, _), ptrs in list(_POOL.items()):
                if tok == self.token:
                    for p in ptrs:
                        self.L.spis_free(self.handle, C.c_void_p(p))
                    ptrs.clear()
            self.L.spis_context_synchronize(self.handle)
            for key in [k for k in _STAGING if k[0] == self.token]:
                for q, _s in _STAGING.pop(key)["slots"]:
                    self.L.spis_host_free(C.c_void_p(q))
            self.L.spis_context_destroy(self.handle)
            self.handle = None


_OPTIONS = {
    "fuse_spmv": (_lib.OPT_FUSE_SPMV, None),
    "orthog": (_lib.OPT_ORTHOG, {"mgs": 0, "cgs2": 1}),
    "con_gram": (_lib.OPT_CON_GRAM, {"generic": 0, "csr": 1, "mfma": 2, "mfma_full": 3}),
    "mgs_chain": (_lib.OPT_MGS_CHAIN, {False: 0, True: 3, "gather0": 1, "aggregator": 2, "pipelined": 3,
                                       "one_reduce": 4}),
    "nt_basis": (_lib.OPT_NT_BASIS, {False: 0, True: 1, "auto": 2}),
    "spmv_pipe": (_lib.OPT_SPMV_PIPE, {"off": 0, "stride": 1, "xcd": 2, "auto": 5, "xcd_natural": 7}),
    "col16": (_lib.OPT_COL16, {False: 0, True: 2, "auto": 1}),
    "dist_mgs": (_lib.OPT_DIST_MGS, {"per_step": 0, "one_reduce": 1}),
    "slab_key": (_lib.OPT_SLAB_KEY, None),
    "gram_inc": (_lib.OPT_GRAM_INC, None),
    "x0_zero_test": (_lib.OPT_X0_ZERO_TEST, None),
    "transpose_pipe": (_lib.OPT_TRANSPOSE_PIPE, None),
    "k2w_small_n": (_lib.OPT_K2W_SMALL_N, int),
    "k2w_fold": (_lib.OPT_K2W_FOLD, None),
    "k2w_tw": (_lib.OPT_K2W_TW, int),
    "k2w_onepass": (_lib.OPT_K2W_ONEPASS, None),
    "store_wt": (_lib.OPT_STORE_WT, int),
}


def set_option(name, value, ctx=None):
    """Per-context solver options (``spis_set_option``, include/spis.h):

    * ``fuse_spmv`` (True): true-residual and Arnoldi SpMVs in one launch (bit-identical);
    * ``orthog`` ("mgs"): "mgs", the reference's modified Gram-Schmidt, or "cgs2", the
      low-synchronisation option (3 reductions per step; not MGS's rounding);
    * ``con_gram`` ("mfma"): how the constraint terms are reduced: "mfma" (f64 matrix cores; a
      symmetric constraint matrix through a slot table of its upper triangle, K7t, any other
      from its CSR, K7m), "mfma_full" (K7m for every matrix), "csr" (the fused reduction without
      matrix cores, K7) or "generic" (SpMM ``M Z`` + tiled Gram);
    * ``mgs_chain`` (True = "pipelined"): each Arnoldi step's MGS chain + normalise as one persistent
      launch, partial dots gathered by a dedicated workgroup ("aggregator") or by workgroup 0
      ("gather0"); "pipelined": each dot product two MGS steps early by the distributive law
      (three exchanges in flight; not MGS's rounding), and beyond its capacity (N > ~1.04M) the
      one-reduce MGS; "one_reduce": two passes per step (every q_l.w and the newest Gram row, then
      the update carrying the previous iteration's GEMV), k <= 32; False = one launch per MGS step;
    * ``nt_basis`` ("auto"): the MGS kernels' basis loads are nontemporal when the matrix and the
      basis exceed the 256 MB Infinity Cache (True: always; False: never), results identical;
    * ``spmv_pipe`` ("auto"): solver SpMV kernels — "xcd" pipelined with an XCD-local walk of
      the row blocks (slab order when the upload found one), "xcd_natural" the same on the natural
      block order, "stride" pipelined grid-stride, "off" unpipelined, "auto" = "xcd" while the
      matrix fits the 256 MB Infinity Cache or has a slab order, else "stride" (rows bit-identical
      in every mode; reduction partials grouped per workgroup);
    * ``col16`` ("auto"): the pipelined SpMV on the 16-bit column copy: "auto" beyond the Infinity
      Cache, True always, False never (rows bit-identical);
    * ``device_ilu`` ("auto"): how a SuperLU ``pre`` (``spilu``/``splu``) is applied — True on
      the device (K8), False by its host ``pre.solve`` through the callback (as the reference
      does), "auto" on the device when the plan's cost model predicts it is faster
      (``DeviceILU.predicted_ms``: shallow level structures; deep dependency chains stay on the
      host, where a sequential sweep is faster than any level-by-level GPU schedule);
    * ``dist_mgs`` ("one_reduce"): several GPUs, MGS's projections in inverse-compact-WY form
      (K2w: 2 all-reduces per Arnoldi step; MGS in exact arithmetic, not its rounding), or
      "per_step" (MGS's j + 2 all-reduces, its rounding);
    * ``slab_key`` (True): matrices uploaded afterwards order the row blocks of a slab by their
      rows' position, so a slab's DoF groups are walked side by side (False: group after group);
    * ``gram_inc``, ``x0_zero_test``, ``transpose_pipe`` (True), ``k2w_small_n`` (-1), ``k2w_fold``
      (True), ``k2w_tw`` (-1), ``k2w_onepass`` (True): A/B switches of parity tests, each
      bitwise-neutral or within roundoff (include/spis.h SPIS_OPT_GRAM_INC ..);
    * ``store_wt`` (1): which kernels store their output vectors write-through, a mask
      (include/spis.h SPIS_OPT_STORE_WT; bitwise-neutral, process-wide);
    * ``verify_uploads`` (True): solver calls that take a SciPy matrix check its full content
      against the cached HBM copy (see :func:`device_matrix`); False trusts identity and buffer
      addresses only (then call :func:`invalidate` after an in-place change)."""
    ctx = ctx or get_context()
    if name == "device_ilu":
        if value not in (True, False, "auto"):
            raise ValueError("device_ilu must be True, False or 'auto'")
        ctx.device_ilu = value
        return
    if name == "verify_uploads":
        global _VERIFY
        _VERIFY = bool(value)
        return
    opt, names = _OPTIONS[name]
    v = int(value) if names is int else names[value] if names is not None else int(bool(value))
    _lib.check(ctx.L.spis_set_option(ctx.handle, opt, v), "spis_set_option")


def _release(ctx, fn_name, handle):
    """Finalizer: release a device object unless its context was already destroyed."""
    if ctx.handle:
        getattr(ctx.L, fn_name)(*([ctx.handle] if fn_name == "spis_free" else []), handle)


_CONTEXTS: dict[int, Context] = {}


def default_device():
    env = os.environ.get("SPIS_DEVICE")
    if env is not None:
        return int(env)
    return 0


def get_context(device=None) -> Context:
    dev = default_device() if device is None else int(device)
    ctx = _CONTEXTS.get(dev)
    if ctx is None:
        ctx = Context(dev)
        _CONTEXTS[dev] = ctx
    return ctx


class DeviceBuffer:
    """Raw HBM allocation (fp64 elements) owned by a context."""

    def __init__(self, ctx: Context, n: int):
        self.ctx = ctx
        self.n = int(n)
        p = C.c_void_p()
        _lib.check(ctx.L.spis_malloc(ctx.handle, 8 * max(self.n, 1), C.byref(p)), "spis_malloc")
        self.ptr = p.value
        self._fin = weakref.finalize(self, _release, ctx, "spis_free", C.c_void_p(self.ptr))

    def upload(self, arr):
        a = np.ascontiguousarray(arr, dtype=np.float64)
        if a.size > self.n:
            raise ValueError("upload larger than buffer")
        _lib.check(self.ctx.L.spis_memcpy_h2d(self.ctx.handle, C.c_void_p(self.ptr), a.ctypes.data_as(C.c_void_p),
                                              8 * a.size), "spis_memcpy_h2d")
        return self

    def download_into(self, out):
        """The first ``len(out)`` entries into the host array ``out`` (returned)."""
        _lib.check(self.ctx.L.spis_memcpy_d2h(self.ctx.handle, out.ctypes.data_as(C.c_void_p), C.c_void_p(self.ptr),
                                              8 * out.size), "spis_memcpy_d2h")
        return out

    def download(self, n=None, pinned=False):
        """The first ``n`` entries as a new host array (``pinned``: in a page-locked buffer from
        :func:`pinned_empty` when one is free or may be made, a pageable one otherwise)."""
        n = self.n if n is None else int(n)
        out = pinned_empty(n) if pinned else None
        if out is None:
            out = np.empty(n, dtype=np.float64)
        _lib.check(self.ctx.L.spis_memcpy_d2h(self.ctx.handle, out.ctypes.data_as(C.c_void_p),
                                              C.c_void_p(self.ptr), 8 * n), "spis_memcpy_d2h")
        return out


# page-locked host buffers for returned iterates: a C3 x (8 MB) comes down at the link's rate in
# one DMA instead of through the runtime's pageable staging.  At most _PINNED_MAX live buffers per
# length; a buffer goes back to its free list when the caller drops the last view of the array
# (so a loop that keeps each result for one step alternates between two), and past the cap (a
# caller that keeps every result) downloads go to ordinary arrays.
_PINNED_FREE: dict = {}
_PINNED_LIVE: dict = {}
_PINNED_MAX = 4


def _pinned_release(n, ptr):
    _PINNED_LIVE[n] = _PINNED_LIVE.get(n, 1) - 1
    if len(_PINNED_FREE.setdefault(n, [])) < _PINNED_MAX:
        _PINNED_FREE[n].append(ptr)
        _PINNED_LIVE[n] += 1  # still allocated, now idle
    else:
        _lib.load_library().spis_host_free(C.c_void_p(ptr))


def pinned_empty(n):
    """A length-``n`` fp64 array in page-locked host memory, or None past the cap."""
    n = int(n)
    free = _PINNED_FREE.get(n)
    ptr = None
    if free:
        try:
            ptr = free.pop()
        except IndexError:
            ptr = None
    if ptr is None:
        if _PINNED_LIVE.get(n, 0) >= _PINNED_MAX:
            return None
        p = C.c_void_p()
        if _lib.load_library().spis_host_alloc(8 * max(n, 1), C.byref(p)) != _lib.OK or not p.value:
            return None
        ptr = p.value
        _PINNED_LIVE[n] = _PINNED_LIVE.get(n, 0) + 1
    arr = np.ctypeslib.as_array((C.c_double * max(n, 1)).from_address(ptr))[:n]
    weakref.finalize(arr.base, _pinned_release, n, ptr)
    return arr


# recycled allocations of solver outputs (DeviceVector.scratch): a solve's result vector is
# dropped by the time the next solve asks for one, and hipMalloc + the zeroing memset cost
# ~20-60 us per solve call (C3: ~2% of a solve).  Reuse is stream-ordered: every libspis
# operation of a context runs on its one stream.
_POOL: dict = {}
_POOL_MAX = 4


def _pool_release(ctx, n, ptr):
    if not ctx.handle:
        return
    lst = _POOL.setdefault((ctx.token, n), [])
    if len(lst) < _POOL_MAX:
        lst.append(ptr)
    else:
        ctx.L.spis_free(ctx.handle, C.c_void_p(ptr))


class DeviceVector(DeviceBuffer):
    """An fp64 vector resident in HBM (length ``n``, room for ``capacity``)."""

    def __init__(self, ctx: Context, n: int, capacity: int | None = None):
        super().__init__(ctx, n if capacity is None else max(n, capacity))
        self.n_valid = int(n)

    @classmethod
    def scratch(cls, ctx: Context, n: int):
        """A length-``n`` vector with unspecified contents, from the context's pool of released
        ones when there is one (for outputs a kernel overwrites whole)."""
        n = int(n)
        lst = _POOL.get((ctx.token, n))
        obj = cls.__new__(cls)
        obj.ctx, obj.n, obj.n_valid = ctx, n, n
        ptr = None
        if lst:
            try:  # a finalizer may run between the test and the pop
                ptr = lst.pop()
            except IndexError:
                ptr = None
        if ptr is not None:
            obj.ptr = ptr
        else:
            p = C.c_void_p()
            _lib.check(ctx.L.spis_malloc(ctx.handle, 8 * max(n, 1), C.byref(p)), "spis_malloc")
            obj.ptr = p.value
        obj._fin = weakref.finalize(obj, _pool_release, ctx, n, obj.ptr)
        return obj

    @classmethod
    def from_host(cls, arr, ctx=None, capacity=None):
        arr = np.ascontiguousarray(arr, dtype=np.float64).reshape(-1)
        ctx = ctx or get_context()
        return cls(ctx, arr.size, capacity).upload(arr)

    def numpy(self):
        return self.download(self.n_valid)

    def __len__(self):
        return self.n_valid

    def __array__(self, dtype=None, copy=None):
        a = self.numpy()
        return a if dtype is None else a.astype(dtype)


class DeviceMatrix:
    """CSR matrix resident in HBM (int32 indices, fp64 values).

    ``halo`` (optional) describes ghost columns for a row-partitioned operator
    (see :mod:`.distributed`)."""

    def __init__(self, ctx: Context, A, halo=None):
        A = _as_csr(A)
        self.ctx = ctx
        self.shape = A.shape
        self.nnz = int(A.nnz)
        h = C.c_void_p()
        halo_p = None
        self._keep = None
        if halo is not None:
            self._keep = halo.ctypes_arrays()
            halo_p = C.byref(halo.desc(self._keep))
        _lib.check(
            ctx.L.spis_csr_upload(
                ctx.handle, A.shape[0], A.shape[1], A.nnz,
                A.indptr.ctypes.data_as(_I32_P), A.indices.ctypes.data_as(_I32_P), A.data.ctypes.data_as(_DOUBLE_P),
                halo_p, C.byref(h),
            ),
            "spis_csr_upload",
        )
        self.handle = h
        self._fin = weakref.finalize(self, _release, ctx, "spis_matrix_destroy", h)
        info = (C.c_int64 * 8)()
        _lib.check(ctx.L.spis_matrix_info(h, info), "spis_matrix_info")
        self.n_blocks = int(info[3])
        self.n_long_rows = int(info[4])
        self.n_ghost = int(info[5])
        self.all_zero = bool(info[6])

    @property
    def n_rows(self):
        return self.shape[0]


def _as_csr(A):
    if not sps.isspmatrix_csr(A) and not isinstance(A, sps.csr_array):
        A = sps.csr_matrix(A)
    data = np.ascontiguousarray(A.data, dtype=np.float64)
    indices = A.indices
    indptr = A.indptr
    if indices.dtype != np.int32 or indptr.dtype != np.int32:
        if A.nnz >= 2 ** 31:
            raise ValueError("nnz >= 2^31 not supported (int32 CSR, as PETSc AIJ)")
        indices = indices.astype(np.int32)
        indptr = indptr.astype(np.int32)
    if data is not A.data or indices is not A.indices or indptr is not A.indptr:
        A = sps.csr_matrix((data, np.ascontiguousarray(indices), np.ascontiguousarray(indptr)), shape=A.shape)
    return A


# ---- upload caches --------------------------------------------------------------------------
_MATRIX_CACHE: dict = {}
_VERIFY = True  # set_option("verify_uploads", ...)
# host threads of the content scans (a persistent pool in libspis, hash.cpp): the C3 operator
# and energy matrix (~0.3 GB) are re-verified within one solve's time at ~16 threads; a GPU box
# grants one process about 16 cores (SPIS_HASH_THREADS overrides the count)
_HASH_THREADS = max(1, int(os.environ.get("SPIS_HASH_THREADS", 0)) or min(16, len(os.sched_getaffinity(0))))
_ASYNC_MIN_BYTES = 1 << 22  # smaller matrices are re-verified inline (a thread hand-off costs more)


def _matrix_key(A):
    return (id(A), A.shape, int(A.nnz), A.data.ctypes.data, A.indices.ctypes.data, A.indptr.ctypes.data)


def content_digest(A):
    """Digest of a sparse matrix's full contents: ``data``, ``indices`` and ``indptr`` (every
    byte, spis_host_hash: ~0.1 ms per 1 MiB per thread), its shape and dtypes."""
    L = _lib.load_library()
    out = C.c_uint64()
    parts = [A.shape, str(A.data.dtype), str(A.indices.dtype), str(A.indptr.dtype)]
    for arr in (A.data, A.indices, A.indptr):
        a = np.ascontiguousarray(arr)
        _lib.check(L.spis_host_hash(C.c_void_p(a.ctypes.data), a.nbytes, _HASH_THREADS, C.byref(out)),
                   "spis_host_hash")
        parts.append(out.value)
    return hash(tuple(parts))


def _nbytes(A):
    if isinstance(A, np.ndarray):
        return A.nbytes
    return A.data.nbytes + A.indices.nbytes + A.indptr.nbytes


def vector_digest(v):
    """Digest of a host vector's full contents (spis_host_hash over every byte) and length."""
    L = _lib.load_library()
    out = C.c_uint64()
    a = np.ascontiguousarray(v, dtype=np.float64)
    _lib.check(L.spis_host_hash(C.c_void_p(a.ctypes.data), a.nbytes, _HASH_THREADS, C.byref(out)), "spis_host_hash")
    return hash((a.size, out.value))


def host_nonzero(v, bitwise=False):
    """``bool(np.any(v))`` for a float vector (``bitwise``: any bit set, so -0.0 counts), on the
    library's scan (stops at the first nonzero entry; an all-zero vector is read on up to
    _HASH_THREADS threads; numpy's ``any`` reads every entry on one)."""
    a = np.asarray(v)
    if a.dtype != np.float64 or not a.flags.c_contiguous or a.ndim != 1:
        return bool(np.any(a.view(np.uint64) if bitwise and a.dtype == np.float64 else a))
    L = _lib.load_library()
    r = C.c_int32(0)
    _lib.check(L.spis_host_nonzero(C.c_void_p(a.ctypes.data), a.size, 1 if bitwise else 0, _HASH_THREADS,
                                   C.byref(r)), "spis_host_nonzero")
    return bool(r.value)


class _Checker:
    """One daemon host thread that re-verifies cached uploads while the solve runs (the hash and
    spis_solve are both ctypes calls, which release the GIL)."""

    def __init__(self):
        self.q: queue.Queue = queue.Queue()
        self.t = threading.Thread(target=self._loop, name="spis-verify", daemon=True)
        self.t.start()

    def _loop(self):
        while True:
            chk = self.q.get()
            try:
                chk.result = chk.digest_fn(chk.A) == chk.digest
            except BaseException as e:  # re-raised by the caller's ok()
                chk.result = e
            chk.done.set()


_CHECKER = None


class PendingCheck:
    """The re-verification of one cached object against its digest, queued on the verifier thread
    when it is made (the digests of a call's operators then overlap its uploads and its solve;
    starting them only at spis_solve measured 0.6 ms of unhidden wait per C3 call on a box whose
    host hashes A and L in 2.7 ms); ``ok()`` waits for it."""

    def __init__(self, A, digest, cache, key, digest_fn=None):
        self.A, self.digest = A, digest
        self.entries = [(cache, key)]  # every cache entry this one digest vouches for
        self.digest_fn = digest_fn or content_digest
        self.result = None
        self.done = threading.Event()
        self.started = False
        self.start()

    def start(self):
        global _CHECKER
        if not self.started:
            self.started = True
            if _CHECKER is None:
                _CHECKER = _Checker()
            _CHECKER.q.put(self)

    def ok(self):
        self.start()
        self.done.wait()
        if isinstance(self.result, BaseException):
            raise self.result
        if not self.result:  # stale: the next lookup rebuilds the entries
            for cache, key in self.entries:
                cache.pop(key, None)
        return self.result


def _cached(cache, key, A, make, checks=None, digest_fn=None, owner=None):
    """Per-object cache entry ``key -> (digest, value)``, evicted when ``A`` is collected (so a later
    object that reuses ``id(A)`` can never hit it).  A hit is re-verified against the full
    contents: inline, or, when ``checks`` is a list and the arrays are large, by a
    :class:`PendingCheck` appended to it, which the caller resolves after the work that used the
    value (solvers._run redoes that work on a stale result)."""
    hit = cache.get(key)
    dig = None
    if hit is not None:
        if not _VERIFY:
            return hit[1]
        if checks is not None and _nbytes(A) >= _ASYNC_MIN_BYTES:
            for chk in checks:  # one digest per object and call (the zero test and the upload of
                # one constraint matrix share it)
                if chk.A is A and chk.digest == hit[0]:
                    chk.entries.append((cache, key))
                    return hit[1]
            checks.append(PendingCheck(A, hit[0], cache, key, digest_fn))
            return hit[1]
        dig = (digest_fn or content_digest)(A)
        if dig == hit[0]:
            return hit[1]
    val = make()
    if hit is None:
        try:
            weakref.finalize(A if owner is None else owner, cache.pop, key, None)
        except TypeError:  # not weak-referenceable: keep until invalidate()
            pass
    cache[key] = ((digest_fn or content_digest)(A) if dig is None else dig, val)
    return val


def device_matrix(A, ctx=None, checks=None) -> DeviceMatrix:
    """HBM copy of SciPy CSR ``A``, cached for the lifetime of ``A`` (keyed on identity and buffer
    addresses) and re-verified against the digest of its full contents on every call — inline,
    or on the verifier thread when ``checks`` (a list the caller resolves) is given."""
    if isinstance(A, DeviceMatrix):
        return A
    ctx = ctx or get_context()
    if not sps.issparse(A) or A.format not in ("csr", "csc"):
        return DeviceMatrix(ctx, A)
    key = _matrix_key(A) + (ctx.device,)
    return _cached(_MATRIX_CACHE, key, A, lambda: DeviceMatrix(ctx, A), checks)


class DeviceILU:
    """Device apply of a SuperLU (incomplete) LU factorisation ``Pr A Pc = L U``: the
    ``pre.solve(vec)`` of ``solvers.py:152-154`` for ``pre = spilu(A, ...)``
    (``swe/TimedSolve.py:23``, ``lkdvRK/Evolve.py:51``) as two sync-free level-blocked triangular
    solves in one launch (K8, ``spis_ilu_*``).  The factorisation stays SuperLU's, on the host."""

    def __init__(self, ctx: Context, lu):
        self.ctx = ctx
        n = int(lu.shape[0])
        self.n = n
        Lf = _as_csr(lu.L.tocsr())
        Uf = _as_csr(lu.U.tocsr())
        Lf.sort_indices()
        Uf.sort_indices()
        pr = np.ascontiguousarray(lu.perm_r, dtype=np.int32)
        pc = np.ascontiguousarray(lu.perm_c, dtype=np.int32)
        h = C.c_void_p()
        _lib.check(
            ctx.L.spis_ilu_create(
                ctx.handle, n, Lf.indptr.ctypes.data_as(_I32_P), Lf.indices.ctypes.data_as(_I32_P),
                Lf.data.ctypes.data_as(_DOUBLE_P), Uf.indptr.ctypes.data_as(_I32_P),
                Uf.indices.ctypes.data_as(_I32_P), Uf.data.ctypes.data_as(_DOUBLE_P),
                pr.ctypes.data_as(_I32_P), pc.ctypes.data_as(_I32_P), C.byref(h)),
            "spis_ilu_create")
        self.handle = h
        self._fin = weakref.finalize(self, _release, ctx, "spis_ilu_destroy", h)
        info = (C.c_int64 * 8)()
        _lib.check(ctx.L.spis_ilu_info(h, info), "spis_ilu_info")
        self.info = {k: int(v) for k, v in zip(
            ("levels_L", "levels_U", "blocks_L", "blocks_U", "steps_L", "steps_U", "nnz_L", "nnz_U"), info)}

    # cost model fitted on MI355X (tools/ilu_sweep.py): the device apply pays ~1.3 us
    # per dependency level plus ~0.32 ns per factor entry; SuperLU's host solve ~2 ns per entry,
    # plus, inside a solve, the callback's two PCIe copies of n doubles and a stream sync
    DEV_US_PER_LEVEL, DEV_NS_PER_NNZ, DEV_US_FIXED = 1.3, 0.32, 20.0
    HOST_NS_PER_NNZ, HOST_US_FIXED, PCIE_GBS = 2.0, 40.0, 25.0

    def predicted_ms(self):
        """(device, host) predicted milliseconds per apply."""
        i = self.info
        nnz = i["nnz_L"] + i["nnz_U"] + 2 * self.n
        dev = (self.DEV_US_PER_LEVEL * (i["levels_L"] + i["levels_U"]) + self.DEV_NS_PER_NNZ * 1e-3 * nnz
               + self.DEV_US_FIXED) * 1e-3
        host = (self.HOST_NS_PER_NNZ * 1e-3 * nnz + self.HOST_US_FIXED
                + 16.0 * self.n / (self.PCIE_GBS * 1e3)) * 1e-3
        return dev, host

    def apply(self, q: DeviceVector, z: DeviceVector):
        _lib.check(self.ctx.L.spis_ilu_apply(self.handle, C.c_void_p(q.ptr), C.c_void_p(z.ptr)), "spis_ilu_apply")
        return z

    def solve(self, b):
        """Host arrays in and out, like ``SuperLU.solve`` (a test/diagnostic convenience)."""
        q = DeviceVector.from_host(np.asarray(b, dtype=np.float64).reshape(-1), ctx=self.ctx)
        z = DeviceVector(self.ctx, self.n)
        return self.apply(q, z).numpy()


def is_superlu(pre):
    return all(hasattr(pre, a) for a in ("L", "U", "perm_r", "perm_c", "solve", "shape"))


_ILU_CACHE: dict = {}
_ILU_CACHE_MAX = 4


def choose_ilu(pre, ctx) -> "DeviceILU | None":
    """The device apply to use for SuperLU object ``pre`` under the context's ``device_ilu``
    option, or None for the host callback."""
    mode = ctx.device_ilu
    if mode is False:
        return None
    d = device_ilu(pre, ctx)
    if mode is True:
        return d
    dev, host = d.predicted_ms()
    return d if dev < host else None


def device_ilu(pre, ctx=None) -> DeviceILU:
    """Device copy of SuperLU object ``pre`` (cached; SuperLU objects take no weak references, so
    the cache holds ``pre`` itself — its id cannot be reused while cached — and keeps the last
    few)."""
    if isinstance(pre, DeviceILU):
        return pre
    ctx = ctx or get_context()
    key = (id(pre), ctx.device)
    hit = _ILU_CACHE.get(key)
    if hit is not None and hit[0] is pre:
        return hit[1]
    d = DeviceILU(ctx, pre)
    while len(_ILU_CACHE) >= _ILU_CACHE_MAX:
        _ILU_CACHE.pop(next(iter(_ILU_CACHE)))
    _ILU_CACHE[key] = (pre, d)
    return d


_ZERO_CACHE: dict = {}


def is_zero_matrix(M, checks=None):
    """Whether a sparse matrix has no nonzero value (the reference wrappers' mass ``0*A`` keeps
    A's pattern with all-zero values).  O(nnz) once per matrix, then cached like
    :func:`device_matrix`: evicted with the object, re-verified against its full contents."""
    if M.nnz == 0:
        return True
    if M.format not in ("csr", "csc"):
        return not np.any(M.data)
    return _cached(_ZERO_CACHE, _matrix_key(M), M, lambda: not host_nonzero(M.data), checks)


def invalidate(A=None):
    """Forget cached uploads and zero tests (of ``A``, or all).  Not needed for correctness (every
    call re-verifies the full contents); it frees the HBM copy early."""
    for cache in (_MATRIX_CACHE, _ZERO_CACHE, _VECTOR_CACHE, _X0_ZERO_CACHE):
        if A is None:
            cache.clear()
            continue
        for key in [k for k in cache if k[0] == id(A)]:
            cache.pop(key, None)


def device_vector(v, ctx=None, capacity=None) -> DeviceVector:
    """HBM copy of a host vector for one call (b, a nonzero x0): its buffer comes from the
    context's pool of released ones (DeviceVector.scratch), so a call pays the copy, not a
    hipMalloc and a hipFree.  From 1 MiB on the array is copied by the host threads into one of
    the context's own page-locked staging buffers (:func:`_stage`) and uploaded from there
    asynchronously (the copy overlaps the call's set-up; the solve on the same stream follows
    it); smaller ones are copied synchronously.  The caller's memory is never page-locked: round
    6 first registered an array seen twice with hipHostRegister, and after such an array was
    freed, copies through the same host pages faulted with an illegal address (intermittently)."""
    if isinstance(v, DeviceVector):
        return v
    if capacity is not None:
        return DeviceVector.from_host(v, ctx=ctx, capacity=capacity)
    a = np.ascontiguousarray(v, dtype=np.float64).reshape(-1)
    ctx = ctx or get_context()
    d = DeviceVector.scratch(ctx, a.size)
    if a.nbytes >= _STAGE_MIN_BYTES and _stage(ctx, d, a):
        return d
    return d.upload(a)


# page-locked staging buffers of the asynchronous uploads (device_vector): two per (context,
# size), used in turn (b and x0 of one call take one each).  A slot is rewritten only after a
# solve on its context has returned since its last upload (the solve's stream follows the
# upload), or after a context synchronize
_STAGE_MIN_BYTES = 1 << 20
_STAGING: dict = {}
_STAGE_MAX = 4  # sizes kept


def _stage(ctx, d, a):
    key = (ctx.token, a.nbytes)
    ent = _STAGING.get(key)
    if ent is None:
        if sum(1 for k in _STAGING if k[0] == ctx.token) >= _STAGE_MAX:
            return False
        L = _lib.load_library()
        slots = []
        for _ in range(2):
            p = C.c_void_p()
            if L.spis_host_alloc(a.nbytes, C.byref(p)) != _lib.OK or not p.value:
                for q, _s in slots:
                    L.spis_host_free(C.c_void_p(q))
                return False
            slots.append([p.value, -1])
        ent = _STAGING[key] = {"slots": slots, "next": 0}
    slot = ent["slots"][ent["next"]]
    ent["next"] ^= 1
    if slot[1] >= ctx.solves:  # its last upload may not have run yet
        ctx.synchronize()
    L = ctx.L
    _lib.check(L.spis_host_copy(C.c_void_p(slot[0]), C.c_void_p(a.ctypes.data), a.nbytes, _HASH_THREADS),
               "spis_host_copy")
    _lib.check(L.spis_memcpy_h2d_async(ctx.handle, C.c_void_p(d.ptr), C.c_void_p(slot[0]), a.nbytes),
               "spis_memcpy_h2d_async")
    slot[1] = ctx.solves
    return True


_VECTOR_CACHE: dict = {}


def _root(a):
    while isinstance(a.base, np.ndarray):
        a = a.base
    return a


def cached_vector(v, ctx=None, checks=None):
    """HBM copy of a host fp64 vector that is part of the problem definition (a constraint's
    ``v``: the wrappers pass the same ``omega`` on every call, e.g. ``swe/LinearSolver.py:28``),
    or None when every entry is zero (np.any's sense: solvers.py drops such a term), cached like
    :func:`device_matrix`: keyed on the array's owner and buffer, evicted with the owner,
    re-verified against a digest of its full contents on every call."""
    if isinstance(v, DeviceVector):
        return v
    ctx = ctx or get_context()
    a = np.asarray(v)

    def make():
        return DeviceVector.from_host(a, ctx=ctx) if host_nonzero(a) else None

    if a.dtype != np.float64 or not a.flags.c_contiguous or a.ndim != 1:
        return make()
    root = _root(a)
    key = (id(root), root.ctypes.data, a.ctypes.data, a.size, ctx.device)
    return _cached(_VECTOR_CACHE, key, a, make, checks, vector_digest, root)


_X0_ZERO_CACHE: dict = {}


def host_x0_zero(a, checks=None):
    """True when the host x0 ``a`` (fp64, 1-D, C-contiguous) is bitwise all +0.0.  The verdict is
    cached like :func:`cached_vector` (keyed on the array's owner and buffer, evicted with it): a
    call handed the same array again takes it from the cache and re-checks it on the verifier
    thread beside the solve (from 4 MiB, a :class:`PendingCheck`; an x0 edited in place since
    discards the run, which then scans inline).  A time-stepping caller's x0 = 0 (8 MB at C3) is
    then read beside the solve, not before it."""

    first = []  # a miss scans once: the verdict is both the value and the entry's "digest"

    def make():
        first.append(not host_nonzero(a, bitwise=True))
        return first[0]

    def verdict(v):
        return first.pop() if first else not host_nonzero(v, bitwise=True)

    root = _root(a)
    key = (id(root), root.ctypes.data, a.ctypes.data, a.size)
    return _cached(_X0_ZERO_CACHE, key, a, make, checks, verdict, root)


_ZERO_VECTORS: dict = {}


def zero_vector(ctx, n) -> DeviceVector:
    """A length-``n`` all-zero HBM vector per context, made once: the x0 of a call whose host x0
    is all zero (the drivers' ``x0 = 0``, e.g. ``swe/TimedSolve.py:37``).  Read-only: no libspis
    entry point writes its x0 argument."""
    key = (ctx.token, int(n))
    z = _ZERO_VECTORS.get(key)
    if z is None:
        if len(_ZERO_VECTORS) >= 4:
            _ZERO_VECTORS.pop(next(iter(_ZERO_VECTORS)))
        z = _ZERO_VECTORS[key] = DeviceVector.from_host(np.zeros(int(n)), ctx=ctx)
    return z


class DeviceConstraint:
    """A class-form constraint ``1/2 X'MX + v.X + c`` (``solvers.py:22-36``) whose operators are
    already resident in HBM: ``M`` a :class:`DeviceMatrix` or None, ``v`` a :class:`DeviceVector`
    or None.  ``solvers.cgmres`` takes it wherever the reference takes a constraint class."""

    def __init__(self, M, v, c):
        self.M, self.v, self.c = M, v, c


def device_constraints(conlist, ctx=None):
    """Upload the operators of reference-form class constraints once (``M`` dropped when it is
    all zeros, ``v`` when it is all zeros, as ``solvers.cgmres`` does per call)."""
    ctx = ctx or get_context()
    out = []
    for con in conlist:
        M = getattr(con, "M", None)
        if M is not None and not isinstance(M, DeviceMatrix):
            Ms = M if sps.issparse(M) else sps.csr_matrix(M)
            M = None if Ms.nnz == 0 or not np.any(Ms.data) else device_matrix(Ms, ctx=ctx)
        v = getattr(con, "v", None)
        if v is not None and not isinstance(v, DeviceVector):
            va = np.asarray(v, dtype=np.float64).reshape(-1)
            v = DeviceVector.from_host(va, ctx=ctx) if np.any(va) else None
        out.append(DeviceConstraint(M, v, float(np.asarray(getattr(con, "c", 0.0)))))
    return out
