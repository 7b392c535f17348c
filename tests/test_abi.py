"""C-ABI: libspis.so loads on CPU, exports every symbol include/spis.h declares,
and the product path fails loudly without a GPU (no CPU fallback)."""
import ctypes as C
import os
import re

import pytest

import structurepreservingiterativesolvers_amd._lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "spis.h")).read()
    return sorted(set(re.findall(r"\b(spis_[a-z0-9_]+)\s*\(", txt)))


def test_header_and_binding_agree():
    declared = header_symbols()
    bound = sorted(name for name, _, _ in L.SIGNATURES)
    assert declared == bound


def test_library_exports_every_symbol():
    lib = C.CDLL(L.LIB_PATH)
    for name in header_symbols():
        assert hasattr(lib, name), name
    assert L.load_library().spis_abi_version() == L.ABI_VERSION


def test_fails_loudly_without_device():
    lib = L.load_library()
    n = C.c_int32(-1)
    assert lib.spis_device_count(C.byref(n)) == 0
    if n.value > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(L.SpisUnavailable):
        L.lib()
    from structurepreservingiterativesolvers_amd import solvers
    import numpy as np
    import scipy.sparse as sps
    with pytest.raises(L.SpisUnavailable):
        solvers.cgmres(sps.identity(4, format="csr"), np.ones(4), np.zeros(4), 2)
    h = C.c_void_p()
    assert lib.spis_context_create(0, C.byref(h)) == L.ERR_HIP
    assert b"no HIP device" in lib.spis_last_error()


def test_missing_library_raises(tmp_path):
    old = L._LIB
    try:
        L._LIB = None
        with pytest.raises(L.SpisUnavailable):
            L.load_library(str(tmp_path / "nope.so"))
    finally:
        L._LIB = old
