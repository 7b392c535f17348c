"""Device ILU plan (K8; csrc/ilu_plan.cpp via the host-only liblsq_host.so), on CPU.

The launch is emulated sequentially in ticket order over the same plan the GPU runs (levels,
solve order, blocks of the LDS window, granule indices, permutations); the emulation fails if
any value would be read before an earlier ticket produced it, i.e. if the GPU launch could wait
on a later ticket.  Its result is compared with SuperLU's own ``pre.solve`` (the reference's
``solvers.py:152-154`` call) on the preconditioners the reference builds (``spilu`` with the
drop tolerances of ``swe/TimedSolve.py:23`` and ``lkdvRK/Evolve.py:51``).  Tolerance: rel 1e-12
(SuperLU's supernodal solve sums in its own order; the factors are identical)."""
import ctypes as C
import os

import numpy as np
import pytest
import scipy.sparse as sps
import scipy.sparse.linalg as spsla

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "structurepreservingiterativesolvers_amd", "liblsq_host.so")
PI, PD = C.POINTER(C.c_int32), C.POINTER(C.c_double)


@pytest.fixture(scope="module")
def host():
    if not os.path.exists(LIB):
        pytest.skip("liblsq_host.so not built (make)")
    L = C.CDLL(LIB)
    L.ilu_plan_emulate.argtypes = [C.c_int64, PI, PI, PD, PI, PI, PD, PI, PI, PD, PD, C.POINTER(C.c_int64),
                                   C.c_char_p, C.c_int]
    return L


def _i(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def _run(host, n, Lf, Uf, pr, pc, q):
    Lf, Uf = sps.csr_matrix(Lf), sps.csr_matrix(Uf)
    Lf.sort_indices()
    Uf.sort_indices()
    arrs = [_i(Lf.indptr), _i(Lf.indices), np.ascontiguousarray(Lf.data, dtype=np.float64),
            _i(Uf.indptr), _i(Uf.indices), np.ascontiguousarray(Uf.data, dtype=np.float64), _i(pr), _i(pc)]
    z = np.zeros(n)
    q = np.ascontiguousarray(q, dtype=np.float64)
    stats = (C.c_int64 * 8)()
    err = C.create_string_buffer(256)
    ptrs = [a.ctypes.data_as(PI if a.dtype == np.int32 else PD) for a in arrs]
    rc = host.ilu_plan_emulate(n, *ptrs, q.ctypes.data_as(PD), z.ctypes.data_as(PD), stats, err, 256)
    return rc, z, list(stats), err.value.decode()


def _problems():
    from structurepreservingiterativesolvers_amd.heat import assembly as ha
    from structurepreservingiterativesolvers_amd.lkdvRK import assembly as ra
    from structurepreservingiterativesolvers_amd.swe import assembly as sa

    return {
        "swe_m16_drop1e-2": (sa.linforms(M=16)[0]["A"], 1e-2),
        "swe_m32_drop1e-4": (sa.linforms(M=32)[0]["A"], 1e-4),
        "lkdvrk_m100_s3_drop1e-4": (ra.linforms(M=100, tstages=3)[0]["A"], 1e-4),
        "heat_m31_drop1e-3": (ha.linforms(M=31)[0]["A"], 1e-3),
    }


@pytest.mark.parametrize("name", list(_problems()))
def test_emulated_apply_matches_superlu_solve(host, name):
    A, drop = _problems()[name]
    P = spsla.spilu(A.tocsc(), drop_tol=drop, fill_factor=10)
    n = A.shape[0]
    rng = np.random.default_rng(0)
    for _ in range(2):
        q = rng.standard_normal(n)
        rc, z, stats, err = _run(host, n, P.L, P.U, P.perm_r, P.perm_c, q)
        assert rc == 0, err
        ref = P.solve(q)
        assert np.linalg.norm(z - ref) <= 1e-12 * np.linalg.norm(ref), name
    lev_l, lev_u, nb_l, nb_u, ns_l, ns_u = stats[:6]
    assert 1 <= lev_l <= n and 1 <= lev_u <= n
    assert nb_l <= ns_l and nb_u <= ns_u
    assert ns_l >= lev_l and ns_u >= lev_u  # every level is at least one step


def test_complete_lu_and_dense_rows(host):
    """splu (no dropping) of a nonsymmetric matrix with a few dense rows/columns (long rows, wide
    and deep levels): the emulated apply solves A z = q."""
    rng = np.random.default_rng(3)
    n = 700
    A = (sps.random(n, n, density=0.004, random_state=4, format="csr") + sps.eye(n) * 5).tolil()
    A[5, :] = rng.standard_normal(n) * 0.01
    A[:, 9] = rng.standard_normal((n, 1)) * 0.01
    A[5, 5] = 7.0
    A = sps.csc_matrix(A)
    P = spsla.splu(A)
    q = rng.standard_normal(n)
    rc, z, _, err = _run(host, n, P.L, P.U, P.perm_r, P.perm_c, q)
    assert rc == 0, err
    assert np.linalg.norm(A @ z - q) <= 1e-10 * np.linalg.norm(q)


def test_chain_spans_many_blocks(host):
    """A bidiagonal factor: n levels of one row, packed 256 rows per block; every block depends
    on its predecessor through a granule."""
    n = 3000
    Lf = sps.eye(n, format="csr") + sps.diags([np.full(n - 1, -0.5)], [-1], format="csr")
    Uf = sps.diags([np.full(n, 2.0), np.full(n - 1, 0.25)], [0, 1], format="csr")
    q = np.random.default_rng(1).standard_normal(n)
    ident = np.arange(n)
    rc, z, stats, err = _run(host, n, Lf, Uf, ident, ident, q)
    assert rc == 0, err
    assert stats[0] == n and stats[2] == (n + 255) // 256
    ref = spsla.spsolve_triangular(sps.csr_matrix(Uf), spsla.spsolve_triangular(sps.csr_matrix(Lf), q, lower=True),
                                   lower=False)
    assert np.linalg.norm(z - ref) <= 1e-13 * np.linalg.norm(ref)


@pytest.mark.parametrize("bad", ["L_diag", "U_diag", "L_upper", "perm"])
def test_plan_rejects_malformed(host, bad):
    n = 20
    Lf = (sps.eye(n, format="csr") + sps.diags([np.full(n - 1, 0.3)], [-1])).tolil()
    Uf = sps.diags([np.full(n, 2.0), np.full(n - 1, 0.1)], [0, 1], format="lil")
    pr = np.arange(n)
    if bad == "L_diag":
        Lf[3, 3] = 2.0
    elif bad == "U_diag":
        Uf[4, 4] = 0.0
    elif bad == "L_upper":
        Lf[2, 7] = 1.0
    else:
        pr = pr.copy()
        pr[1] = 0
    rc, _, _, err = _run(host, n, Lf, Uf, pr, np.arange(n), np.ones(n))
    assert rc != 0 and err
