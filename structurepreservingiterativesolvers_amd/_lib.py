"""ctypes binding of ``libspis.so`` (C-ABI declared in ``include/spis.h``).

The product path has no CPU fallback: if the library is missing, was built for
another ABI, or no HIP device is visible, :func:`lib` raises
:class:`SpisUnavailable` with the reason.  Build with ``make`` (or
``__graft_entry__.build()``); the ``.so`` lives next to this file.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SPIS_LIBRARY", os.path.join(_HERE, "libspis.so"))
ABI_VERSION = 1

# status codes (spis_status)
OK, ERR_ARG, ERR_HIP, ERR_RCCL, ERR_ALLOC, ERR_CALLBACK, ERR_STATE = range(7)
# methods / branches / events / messages
CGMRES, GMRES, CGMRES_P = 0, 1, 2
BRANCH_UNCON, BRANCH_CON, BRANCH_FALLBACK = 0, 1, 2
EV_BREAKDOWN, EV_LS_MESSAGE, EV_NAN, EV_VIOLATION, EV_FALLBACK = 1, 2, 4, 8, 16
PROF_SPMV, PROF_MGS, PROF_GEMV, PROF_SPMV_RES, PROF_SPMV_DUAL = range(5)
PROF_KINDS = 5
# spis_option (include/spis.h)
OPT_FUSE_SPMV = 1
OPT_ORTHOG = 4
OPT_CON_GRAM = 5
OPT_MGS_CHAIN = 6
OPT_SPMV_PIPE = 8
OPT_NT_BASIS = 10
OPT_COL16 = 11
OPT_DIST_MGS = 12
OPT_SLAB_KEY = 16
OPT_GRAM_INC = 17
OPT_X0_ZERO_TEST = 18
OPT_TRANSPOSE_PIPE = 19
OPT_STORE_WT = 24
OPT_K2W_SMALL_N = 20
OPT_K2W_FOLD = 21
OPT_K2W_TW = 22
OPT_K2W_ONEPASS = 23
MESSAGES = {
    0: "Optimization terminated successfully",
    2: "More equality constraints than independent variables",
    6: "Singular matrix C in LSQ subproblem",
    9: "Iteration limit reached",
}


class SpisError(RuntimeError):
    """A libspis call returned a non-zero status."""

    def __init__(self, code, where, msg):
        super().__init__(f"{where} failed with status {code}: {msg}")
        self.code = code


class SpisUnavailable(ImportError):
    """libspis.so cannot be used (not built, wrong ABI, or no MI355X visible)."""


class HaloDesc(C.Structure):
    _fields_ = [
        ("n_ghost", C.c_int32),
        ("n_neighbors", C.c_int32),
        ("neighbors", C.POINTER(C.c_int32)),
        ("send_counts", C.POINTER(C.c_int32)),
        ("send_idx", C.POINTER(C.c_int32)),
        ("recv_counts", C.POINTER(C.c_int32)),
    ]


class ConstraintDesc(C.Structure):
    _fields_ = [("M", C.c_void_p), ("v_dev", C.c_void_p), ("c", C.c_double)]


PRECOND_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int64)
# spis_host_coll_fn (spis_comm_init_host): (user, op, buf, count, n_neighbors, neighbors,
# send_counts, recv_counts, recv)
HOST_COLL_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int32, C.POINTER(C.c_double), C.c_int64, C.c_int32,
                           C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_double))
COLL_ALLREDUCE, COLL_EXCHANGE = 0, 1
CONLS_FN = C.CFUNCTYPE(
    C.c_int, C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.POINTER(C.c_double), C.c_double,
    C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_int32), C.POINTER(C.c_int32),
    C.POINTER(C.c_int32),
)


class SolveOpts(C.Structure):
    _fields_ = [
        ("method", C.c_int32),
        ("k", C.c_int32),
        ("tol", C.c_double),
        ("contol", C.c_double),
        ("timing", C.c_int32),
        ("n_constraints", C.c_int32),
        ("constraints", C.POINTER(ConstraintDesc)),
        ("pre_matrix", C.c_void_p),
        ("pre_fn", PRECOND_FN),
        ("pre_user", C.c_void_p),
        ("conls_fn", CONLS_FN),
        ("conls_user", C.c_void_p),
        ("pre_ilu", C.c_void_p),
    ]


class SolveOut(C.Structure):
    _fields_ = [
        ("steps", C.c_int32),
        ("n_res", C.c_int32),
        ("res_host", C.POINTER(C.c_double)),
        ("y_host", C.POINTER(C.c_double)),
        ("branch_host", C.POINTER(C.c_int32)),
        ("events_host", C.POINTER(C.c_int32)),
        ("msg_host", C.POINTER(C.c_int32)),
        ("stamps_host", C.POINTER(C.c_double)),
        ("x_final_dev", C.c_void_p),
        ("x_final_host", C.c_void_p),
        ("x_host_ready", C.c_int32),
    ]


# (name, restype, argtypes) — every symbol include/spis.h declares
_VP, _I32, _I64, _D = C.c_void_p, C.c_int32, C.c_int64, C.c_double
_PD, _PI32, _PI64 = C.POINTER(C.c_double), C.POINTER(C.c_int32), C.POINTER(C.c_int64)
SIGNATURES = [
    ("spis_abi_version", C.c_int, []),
    ("spis_last_error", C.c_char_p, []),
    ("spis_device_count", C.c_int, [_PI32]),
    ("spis_context_create", C.c_int, [_I32, C.POINTER(_VP)]),
    ("spis_context_destroy", C.c_int, [_VP]),
    ("spis_context_synchronize", C.c_int, [_VP]),
    ("spis_context_stream", C.c_int, [_VP, C.POINTER(_VP)]),
    ("spis_host_hash", C.c_int, [_VP, _I64, _I32, C.POINTER(C.c_uint64)]),
    ("spis_host_nonzero", C.c_int, [_VP, _I64, _I32, _I32, _PI32]),
    ("spis_host_copy", C.c_int, [_VP, _VP, _I64, _I32]),
    ("spis_host_isa_ok", C.c_int, []),
    ("spis_profile_enable", C.c_int, [_VP, _I32]),
    ("spis_profile_read", C.c_int, [_VP, _PD, _PI64]),
    ("spis_spmv_bench", C.c_int, [_VP, _VP, _I32, _I32, _I32, _PD]),
    ("spis_set_option", C.c_int, [_VP, _I32, _I64]),
    ("spis_comm_unique_id", C.c_int, [C.POINTER(C.c_uint8)]),
    ("spis_comm_init", C.c_int, [_VP, _I32, _I32, C.POINTER(C.c_uint8)]),
    ("spis_comm_allreduce_sum", C.c_int, [_VP, _VP, _I64]),
    ("spis_comm_barrier", C.c_int, [_VP]),
    ("spis_comm_size", C.c_int, [_VP, _PI32, _PI32]),
    ("spis_comm_init_host", C.c_int, [_VP, _I32, _I32, HOST_COLL_FN, _VP]),
    ("spis_csr_upload", C.c_int, [_VP, _I64, _I64, _I64, _PI32, _PI32, _PD, C.POINTER(HaloDesc), C.POINTER(_VP)]),
    ("spis_matrix_destroy", C.c_int, [_VP]),
    ("spis_matrix_info", C.c_int, [_VP, _PI64]),
    ("spis_matrix_set_global", C.c_int, [_VP, _PI64, _I32]),
    ("spis_ilu_create", C.c_int, [_VP, _I64, _PI32, _PI32, _PD, _PI32, _PI32, _PD, _PI32, _PI32, C.POINTER(_VP)]),
    ("spis_ilu_apply", C.c_int, [_VP, _VP, _VP]),
    ("spis_ilu_info", C.c_int, [_VP, _PI64]),
    ("spis_ilu_destroy", C.c_int, [_VP]),
    ("spis_malloc", C.c_int, [_VP, _I64, C.POINTER(_VP)]),
    ("spis_free", C.c_int, [_VP, _VP]),
    ("spis_memcpy_h2d", C.c_int, [_VP, _VP, _VP, _I64]),
    ("spis_memcpy_d2h", C.c_int, [_VP, _VP, _VP, _I64]),
    ("spis_host_alloc", C.c_int, [_I64, C.POINTER(_VP)]),
    ("spis_host_free", C.c_int, [_VP]),
    ("spis_host_register", C.c_int, [_VP, _I64]),
    ("spis_host_unregister", C.c_int, [_VP]),
    ("spis_memcpy_h2d_async", C.c_int, [_VP, _VP, _VP, _I64]),
    ("spis_copy_to_host", C.c_int, [_VP, _PD, _VP, _I64]),
    ("spis_spmv", C.c_int, [_VP, _VP, _VP, _VP]),
    ("spis_residual_norm", C.c_int, [_VP, _VP, _VP, _VP, _PD]),
    ("spis_dot", C.c_int, [_VP, _I64, _VP, _VP, _PD]),
    ("spis_nrm2", C.c_int, [_VP, _I64, _VP, _PD]),
    ("spis_axpy", C.c_int, [_VP, _I64, _D, _VP, _VP]),
    ("spis_gemv", C.c_int, [_VP, _I64, _I32, _VP, _I64, _PD, _VP, _VP]),
    ("spis_gram", C.c_int, [_VP, _I64, _I32, C.POINTER(_VP), _I32, C.POINTER(_VP), _PD]),
    ("spis_constraint_terms", C.c_int, [_VP, C.POINTER(ConstraintDesc), _I64, _I32, _VP, _I64, _VP, _PD, _PD, _PD]),
    ("spis_solve", C.c_int, [_VP, _VP, _VP, _VP, C.POINTER(SolveOpts), C.POINTER(SolveOut), C.POINTER(_VP)]),
    ("spis_workspace_iterate", C.c_int, [_VP, _I32, _VP]),
    ("spis_workspace_basis", C.c_int, [_VP, _I32, _PD]),
    ("spis_workspace_hessenberg", C.c_int, [_VP, _I32, _PD]),
    ("spis_workspace_constraint_terms", C.c_int, [_VP, _I32, C.POINTER(C.c_int32), _PD, _PD, _PD]),
    ("spis_workspace_release", C.c_int, [_VP]),
]

_LIB = None


def load_library(path=LIB_PATH):
    """Load libspis.so and bind every exported symbol (no device needed)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise SpisUnavailable(
            f"libspis.so not found at {path}: build it with `make` (hipcc --offload-arch=gfx950); "
            "there is no CPU fallback for the solver path"
        )
    try:
        lib = C.CDLL(path)
    except OSError as e:  # pragma: no cover - depends on the ROCm install
        raise SpisUnavailable(f"cannot load {path}: {e}") from e
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.spis_abi_version() != ABI_VERSION:
        raise SpisUnavailable(f"{path}: ABI {lib.spis_abi_version()} != expected {ABI_VERSION}")
    if not lib.spis_host_isa_ok():
        raise SpisUnavailable(f"{path}: its host least squares is built for x86-64-v3 (AVX2, FMA, BMI2), which "
                              "this CPU lacks; rebuild with `make LSQFLAGS=-ffp-contract=off` (INTEGRATION.md)")
    _LIB = lib
    return lib


def check(status, where):
    if status != OK:
        msg = _LIB.spis_last_error().decode(errors="replace") if _LIB else "?"
        raise SpisError(status, where, msg)


def lib():
    """The bound library, with a HIP device guaranteed visible."""
    L = load_library()
    n = C.c_int32(0)
    check(L.spis_device_count(C.byref(n)), "spis_device_count")
    if n.value < 1:
        raise SpisUnavailable("no HIP device visible: the spis solver path runs only on an MI355X (gfx950)")
    return L


def profile_read(L, handle):
    """(total ms, launch count) per SPIS_PROF_* kind since spis_profile_enable."""
    ms = (C.c_double * PROF_KINDS)()
    cnt = (C.c_int64 * PROF_KINDS)()
    check(L.spis_profile_read(handle, ms, cnt), "spis_profile_read")
    return list(ms), list(cnt)
