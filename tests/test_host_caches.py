"""Host-side upload / zero-test caches (device.py): keyed on identity + buffer addresses + a
sampled content fingerprint, evicted with the object.  CPU only: no upload happens here."""
import gc

import numpy as np
import scipy.sparse as sps

from structurepreservingiterativesolvers_amd import device


def _mat(seed, zero=False):
    rng = np.random.default_rng(seed)
    A = sps.random(500, 500, density=0.02, random_state=rng, format="csr") + sps.identity(500, format="csr")
    A = sps.csr_matrix(A)
    return 0 * A if zero else A


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


def test_zero_cache_sees_in_place_change_at_sampled_entry():
    M = _mat(1, zero=True)
    assert device.is_zero_matrix(M)
    M.data[0] = 1.0  # entry 0 is always sampled
    assert not device.is_zero_matrix(M)
    M.data[0] = 0.0
    assert device.is_zero_matrix(M)


def test_invalidate_forgets_entries():
    M = _mat(2, zero=True)
    assert device.is_zero_matrix(M)
    device.invalidate(M)
    assert device._matrix_key(M) not in device._ZERO_CACHE
    assert device.is_zero_matrix(M)
    device.invalidate()
    assert not device._ZERO_CACHE


def test_fingerprint_samples_every_size():
    for n in (1, 7, 5000, 100_000):
        A = sps.csr_matrix(sps.diags([np.arange(1.0, n + 1)], [0]) + sps.eye(n, k=1))
        f = device.fingerprint(A)
        A.data[:] += 1.0
        assert device.fingerprint(A) != f
