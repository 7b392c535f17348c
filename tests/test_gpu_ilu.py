"""GPU: the device ILU apply (K8, ``spis_ilu_*``) against SuperLU's own ``pre.solve`` — the call
the reference makes at ``solvers.py:152-154`` — and the preconditioned solvers with the device
apply against the same solvers with the host callback and against the oracle.

Tolerances: apply rel 1e-12 (same factors; SuperLU's supernodal solve and the row-oriented
device solve sum in different orders).  Preconditioned solver iterates: rel 1e-8 per iterate
(tests/test_gpu_parity.py's iterate bound)."""
import time

import numpy as np
import pytest
import scipy.sparse as sps
import scipy.sparse.linalg as spsla

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def spis():
    import structurepreservingiterativesolvers_amd as pkg
    from structurepreservingiterativesolvers_amd import _lib

    _lib.lib()
    return pkg


def _cases():
    from structurepreservingiterativesolvers_amd.heat import assembly as ha
    from structurepreservingiterativesolvers_amd.lkdvRK import assembly as ra
    from structurepreservingiterativesolvers_amd.swe import assembly as sa

    return {
        "swe_m16_drop1e-2": lambda: (sa.linforms(M=16)[0]["A"], 1e-2),
        "swe_m64_drop1e-2": lambda: (sa.linforms(M=64)[0]["A"], 1e-2),
        "swe_m32_drop1e-4": lambda: (sa.linforms(M=32)[0]["A"], 1e-4),
        "lkdvrk_m200_s3_drop1e-4": lambda: (ra.linforms(M=200, tstages=3)[0]["A"], 1e-4),
        "lkdvrk_m50_s2_drop1e-4": lambda: (ra.linforms(M=50, tstages=2)[0]["A"], 1e-4),
        "heat_m31_drop1e-3": lambda: (ha.linforms(M=31)[0]["A"], 1e-3),
    }


@pytest.mark.parametrize("name", list(_cases()))
def test_device_ilu_apply_matches_superlu(spis, name):
    from structurepreservingiterativesolvers_amd import device

    A, drop = _cases()[name]()
    P = spsla.spilu(A.tocsc(), drop_tol=drop, fill_factor=10)
    d = device.DeviceILU(device.get_context(), P)
    rng = np.random.default_rng(0)
    for _ in range(5):  # repeated applies: granules and ticket re-initialised every call
        q = rng.standard_normal(A.shape[0])
        ref = P.solve(q)
        z = d.solve(q)
        assert np.linalg.norm(z - ref) <= 1e-12 * np.linalg.norm(ref), (name, d.info)


def test_device_ilu_complete_lu_solves_system(spis):
    from structurepreservingiterativesolvers_amd import device

    rng = np.random.default_rng(3)
    n = 5000
    A = (sps.random(n, n, density=0.002, random_state=4, format="csr") + sps.eye(n) * 5).tocsc()
    P = spsla.splu(A)
    d = device.DeviceILU(device.get_context(), P)
    q = rng.standard_normal(n)
    z = d.solve(q)
    assert np.linalg.norm(A @ z - q) <= 1e-10 * np.linalg.norm(q)
    np.testing.assert_allclose(z, P.solve(q), rtol=0, atol=1e-12 * np.abs(z).max())


def test_device_ilu_long_chain(spis):
    """n one-row levels (bidiagonal factors): every block hands off to the next."""
    from structurepreservingiterativesolvers_amd import device

    n = 20000
    A = sps.diags([np.full(n, 4.0), np.full(n - 1, -1.0), np.full(n - 1, -1.5)], [0, -1, 1], format="csc")
    P = spsla.splu(A, permc_spec="NATURAL", diag_pivot_thresh=0.0)
    d = device.DeviceILU(device.get_context(), P)
    assert d.info["levels_L"] == n
    q = np.random.default_rng(2).standard_normal(n)
    z = d.solve(q)
    assert np.linalg.norm(A @ z - q) <= 1e-12 * np.linalg.norm(q)


def test_apply_rejects_alias_and_bad_factors(spis):
    from structurepreservingiterativesolvers_amd import _lib, device

    ctx = device.get_context()
    A = sps.diags([np.full(50, 3.0), np.full(49, 1.0)], [0, 1], format="csc")
    d = device.DeviceILU(ctx, spsla.splu(A))
    v = device.DeviceVector.from_host(np.ones(50), ctx=ctx)
    with pytest.raises(_lib.SpisError):
        d.apply(v, v)

    class Fake:
        shape = (50, 50)
        L = sps.eye(50, format="csc") * 2.0  # not unit lower
        U = sps.eye(50, format="csc")
        perm_r = np.arange(50)
        perm_c = np.arange(50)

        def solve(self, b):
            return b

    with pytest.raises(_lib.SpisError):
        device.DeviceILU(ctx, Fake())


def _swe_timed(M):
    from structurepreservingiterativesolvers_amd.swe import assembly as sa

    params, prob = sa.linforms(M=M)
    pre = spsla.spilu(params["A"].tocsc(), drop_tol=1e-2, fill_factor=10)  # swe/TimedSolve.py:23
    return params, prob, pre


@pytest.mark.parametrize("wrapper", ["gmresWrapper", "cgmresWrapper"])
def test_swe_timedsolve_device_ilu_vs_host_callback_and_oracle(spis, wrapper):
    """swe/TimedSolve.py:18-40 at M=16: gmres and cgmres with the spilu preconditioner; the device
    apply against the host pre.solve callback and against the oracle."""
    from oracle import cgmres_port as port
    from structurepreservingiterativesolvers_amd import device
    from structurepreservingiterativesolvers_amd.swe import LinearSolver as ls

    params, prob, pre = _swe_timed(16)
    x0 = np.zeros_like(params["b"])
    fn = getattr(ls, wrapper)
    device.set_option("device_ilu", True)
    xd, dd = fn(params, x0=x0, k=20, tol=1e-7, pre=pre)
    try:
        device.set_option("device_ilu", False)
        xh, dh = fn(params, x0=x0, k=20, tol=1e-7, pre=pre)
    finally:
        device.set_option("device_ilu", "auto")
    if wrapper == "gmresWrapper":
        xr, dr = port.gmres(params["A"], params["b"], x0, 20, tol=1e-7, pre=pre)
    else:
        xr, dr = port.cgmres(params["A"], params["b"], x0, 20, tol=1e-7,
                             conlist=ls.constraints(params, x0), pre=pre)
    assert dd["steps"] == dh["steps"] == dr["steps"]
    for i in range(1, dd["steps"] + 1):
        ref = np.asarray(dr["x"][i])
        for d in (dd, dh):
            assert np.linalg.norm(np.asarray(d["x"][i]) - ref) <= 1e-8 * np.linalg.norm(ref), i
    # residuals to the iterate bound (1e-8 relative, scaled by r0): the constrained last step's
    # residual sits at 1e-9 r0 and moves with its SLSQP solution
    np.testing.assert_allclose(dd["res"], dr["res"], rtol=1e-7, atol=1e-8 * dr["res"][0])


def test_auto_policy_picks_device_for_shallow_and_host_for_deep_chains(spis):
    """device_ilu="auto": swe's spilu (~200 levels for 2e5 rows) goes to the device, lkdvRK's
    (levels ~ 0.6 n: a near-sequential chain) stays with SuperLU's host solve."""
    from structurepreservingiterativesolvers_amd import device
    from structurepreservingiterativesolvers_amd.lkdvRK import assembly as ra

    ctx = device.get_context()
    _, _, pre = _swe_timed(128)
    assert device.choose_ilu(pre, ctx) is not None
    A = ra.linforms(M=2000, tstages=3)[0]["A"]
    pre_rk = spsla.spilu(A.tocsc(), drop_tol=1e-4, fill_factor=10)
    assert device.choose_ilu(pre_rk, ctx) is None
    device.set_option("device_ilu", True)
    try:
        assert device.choose_ilu(pre_rk, ctx) is not None
    finally:
        device.set_option("device_ilu", "auto")


def test_device_ilu_speed_vs_host_solve(spis, capsys):
    """Report (no assertion on speed): one device apply vs SuperLU's host solve at swe M=128."""
    from structurepreservingiterativesolvers_amd import device

    params, _, pre = _swe_timed(128)
    ctx = device.get_context()
    d = device.device_ilu(pre, ctx)
    n = params["A"].shape[0]
    q = device.DeviceVector.from_host(np.random.default_rng(0).standard_normal(n), ctx=ctx)
    z = device.DeviceVector(ctx, n)
    for _ in range(3):
        d.apply(q, z)
    t = time.perf_counter()
    for _ in range(20):
        d.apply(q, z)
    t_dev = (time.perf_counter() - t) / 20
    qh = q.numpy()
    t = time.perf_counter()
    for _ in range(5):
        ref = pre.solve(qh)
    t_host = (time.perf_counter() - t) / 5
    assert np.linalg.norm(z.numpy() - ref) <= 1e-12 * np.linalg.norm(ref)
    with capsys.disabled():
        print(f"\nswe M=128 n={n} ILU apply: device {t_dev * 1e3:.3f} ms, host SuperLU {t_host * 1e3:.3f} ms, "
              f"plan {d.info}")
