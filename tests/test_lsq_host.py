"""Host small-LS (csrc/lsq.cpp, via the host-only liblsq_host.so) against the
reference's own least-squares solutions: for every golden cgmres run, the
oracle (bit-exact with the reference) rebuilds H and the constraint terms of
each iteration, and the Givens / Newton-KKT solutions are compared with the
``y`` the reference's SLSQP returned (logged in the fixture)."""
import ctypes as C
import os

import numpy as np
import pytest

from _golden import Case, names
from oracle.cgmres_port import ConstraintTerms, _Arnoldi

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "structurepreservingiterativesolvers_amd", "liblsq_host.so")
PD = C.POINTER(C.c_double)


@pytest.fixture(scope="module")
def lsq():
    if not os.path.exists(LIB):
        pytest.skip("liblsq_host.so not built (make)")
    L = C.CDLL(LIB)
    L.lsq_givens_solve.argtypes = [C.c_int, PD, C.c_double, PD]
    L.lsq_kkt_solve.argtypes = [C.c_int, PD, C.c_double, C.c_int, PD, PD, PD, PD, PD, C.POINTER(C.c_int),
                                C.POINTER(C.c_int)]
    L.lsq_con_value.argtypes = [C.c_int, C.c_double, PD, PD, PD]
    L.lsq_con_value.restype = C.c_double
    return L


def _p(a):
    return np.ascontiguousarray(a, dtype=np.float64).ctypes.data_as(PD)


def givens(L, Hj, beta):
    p = Hj.shape[1]
    y = np.zeros(p)
    Hc = np.asfortranarray(Hj)
    L.lsq_givens_solve(p, Hc.ctypes.data_as(PD), beta, y.ctypes.data_as(PD))
    return y


def kkt(L, Hj, beta, terms, y0):
    p = Hj.shape[1]
    m = len(terms)
    t0 = np.array([t[0] for t in terms])
    t1 = np.concatenate([t[1] for t in terms]) if m else np.zeros(1)
    t2 = np.concatenate([np.ascontiguousarray(t[2]).ravel() for t in terms]) if m else np.zeros(1)
    y = np.zeros(p)
    msg, it = C.c_int(), C.c_int()
    Hc = np.asfortranarray(Hj)
    L.lsq_kkt_solve(p, Hc.ctypes.data_as(PD), beta, m, _p(t0), _p(t1), _p(t2), _p(y0), y.ctypes.data_as(PD),
                    C.byref(msg), C.byref(it))
    return y, msg.value, it.value


CGMRES_CASES = [n for n in names() if Case(n).solver == "cgmres" and Case(n).meta["problem"] not in ("lkdvRK", "edge")]


@pytest.mark.parametrize("name", CGMRES_CASES)
def test_givens_and_kkt_match_reference_slsqp(lsq, name):
    case = Case(name)
    st = _Arnoldi(case.A, case.b, case.x0, case.k, case.preconditioner())
    cons = case.conlist()
    j = -1
    prev_y = None
    checked = 0
    for i, (p, nc, msg) in enumerate(zip(case.calls_p, case.calls_ncons, case.calls_msg)):
        while j < p - 1:
            j += 1
            st.extend(j)
        Hj = st.H[: p + 1, :p]
        yref = case.calls_y[i, :p]
        scale = max(1.0, np.abs(yref).max())
        if nc == 0:
            y = givens(lsq, Hj, st.beta)
            # SLSQP stops at ftol=1e-24 on ||.||^2: early iterates agree to ~1e-10
            assert np.abs(y - yref).max() <= 1e-7 * scale, (j, np.abs(y - yref).max())
        else:
            Z = st.basis(p - 1)
            terms = []
            for c in cons:
                t = ConstraintTerms(c, case.x0, Z)
                terms.append((t.term0, t.term1, t.term2))
            y0 = np.zeros(p)
            if prev_y is not None:
                y0[:-1] = prev_y[: p - 1]
            y, m, it = kkt(lsq, Hj, st.beta, terms, y0)
            if msg == "More equality constraints than independent variables":
                assert m == 2 and np.array_equal(y, y0)
            elif msg == "Optimization terminated successfully":
                assert m == 0, (j, m)
                assert np.abs(y - yref).max() <= 1e-8 * scale, (j, np.abs(y - yref).max())
                # signed checker passes (solvers.py:267): computed values <= ctol
                for t0, t1, t2 in terms:
                    assert lsq.lsq_con_value(p, t0, _p(t1), _p(t2), _p(y)) <= 1e-12
        prev_y = yref
        checked += 1
    assert checked > 0


def test_givens_matches_lstsq_random(lsq):
    rng = np.random.default_rng(0)
    for p in (1, 2, 5, 17, 40):
        H = np.triu(rng.normal(size=(p + 1, p)), -1) + 4.0 * np.eye(p + 1, p)
        beta = 3.0
        rhs = np.zeros(p + 1)
        rhs[0] = beta
        y = givens(lsq, H, beta)
        yref = np.linalg.lstsq(H, rhs, rcond=None)[0]
        np.testing.assert_allclose(y, yref, rtol=1e-10, atol=1e-12)


def test_kkt_overconstrained_returns_initial_guess(lsq):
    """SLSQP exit mode 2 (m > p) leaves x at the initial guess (fixture lkdv_m50_overconstrained)."""
    H = np.array([[2.0], [1.0]])
    terms = [(1.0, np.array([1.0]), np.array([[0.0]]))] * 2
    y, msg, _ = kkt(lsq, H, 1.0, terms, np.array([0.25]))
    assert msg == 2 and y[0] == 0.25


def test_kkt_rejects_constrained_maximum(lsq):
    """Newton on the KKT system converges to any stationary point.  Warm-started next to the
    constrained MAXIMUM of ||(2, 0) - y||^2 on the unit circle (y = (-1, 0), multiplier -3,
    reduced Hessian negative), kkt_newton must reject it by its second-order test and return
    the minimum (1, 0) that SLSQP finds, with a success message."""
    import scipy.optimize as spo

    H = np.array([[1.0, 0.0], [0.0, 1.0], [0.0, 0.0]])
    terms = [(-1.0, np.zeros(2), np.eye(2))]
    y0 = np.array([-1.0, 0.01])
    y, msg, _ = kkt(lsq, H, 2.0, terms, y0)
    assert msg == 0
    np.testing.assert_allclose(y, [1.0, 0.0], atol=1e-12)
    rhs = np.array([2.0, 0.0, 0.0])
    sol = spo.minimize(lambda z: np.sum((rhs - H @ z) ** 2), y0, jac=lambda z: -2 * H.T @ (rhs - H @ z),
                       constraints=[{"type": "eq", "fun": lambda z: z @ z - 1.0, "jac": lambda z: 2 * z}],
                       method="SLSQP", options={"ftol": 1e-24, "maxiter": 1000})
    np.testing.assert_allclose(y, sol.x, atol=1e-8)


def test_kkt_lkdvrk_gl3_final_step_matches_slsqp(lsq):
    """The constrained step of config C4's shape (lkdvRK GL(3), 3 lifted invariants) at M=400:
    the oracle (the reference's arithmetic) builds H and the constraint terms of step j = 29,
    and the Newton-KKT solution matches the reference's SLSQP on those identical inputs.  This
    step is degenerate: the mass constraint's term0 is exactly 0 and its term1 is roundoff
    (|term1| ~ 4e-15, the Krylov vectors carry no mass), so its Jacobian row is noise and the
    solution's dependence on roundoff is the reference's own; on identical
    inputs the two solvers still agree to ~1e-10."""
    from oracle.cgmres_port import _slsqp
    from structurepreservingiterativesolvers_amd.lkdvRK import LinearSolver as rk_ls
    from structurepreservingiterativesolvers_amd.lkdvRK import assembly as ra

    dic, prob = ra.linforms(M=400, tstages=3)
    x0 = np.zeros_like(dic["b"])
    cons = rk_ls.constraints(dic, prob)
    k = 30
    st = _Arnoldi(dic["A"], dic["b"], x0, k, None)
    yk = None
    for j in range(k):
        st.extend(j)
        _, func, jac = st.ls_objective(j)
        y0 = np.zeros(j + 1)
        if j:
            y0[:-1] = yk
        if j < k - 1:  # the reference's unconstrained steps (its warm starts, :225-235)
            yk = _slsqp(func, y0, jac, [], 1e-24).x
    Z = st.basis(k - 1)
    terms = [ConstraintTerms(c, x0, Z) for c in cons]
    sol = _slsqp(func, y0, jac, [t.as_slsqp() for t in terms], 1e-24)
    assert sol.message == "Optimization terminated successfully"
    y, msg, _ = kkt(lsq, st.H[: k + 1, :k], st.beta, [(t.term0, t.term1, t.term2) for t in terms], y0)
    assert msg == 0
    assert np.linalg.norm(y - sol.x) <= 1e-9 * np.linalg.norm(sol.x)
    for t in terms:  # the signed checker passes (solvers.py:267)
        assert lsq.lsq_con_value(k, t.term0, _p(t.term1), _p(t.term2), _p(y)) <= 1e-12
    assert func(y) <= func(sol.x) * (1 + 1e-9)
    assert abs(terms[0].term0) == 0.0 and np.linalg.norm(terms[0].term1) < 1e-12  # the degeneracy


def test_kkt_singular_constraint_gradient_exits_as_slsqp(lsq):
    """Config C4's forced constrained step as the device solver saw it (H, beta, warm start and
    the three reduced constraints dumped by tools/dump_kkt_case.py from a GPU run): the mass
    constraint's gradient is roundoff (|term1| ~ 1e-18, term0 ~ 7e-15), so SLSQP's first LSQ
    subproblem stops with "Singular matrix C in LSQ subproblem" at the warm start.  The KKT solve
    must exit the same way (message 6, y = y0) instead of running both Newton starts to the
    iteration limit; the reference then falls back (constraint_checker > ctol), as the oracle
    does at this size."""
    import os
    from oracle.cgmres_port import _slsqp

    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "kkt_cases", "kkt_c4_final_step.npz"))
    H, beta, y0 = z["H"], float(z["beta"]), z["y0"]
    k = H.shape[1]
    terms = [(z["t0"][i], z["t1"][i], z["t2"][i]) for i in range(len(z["t0"]))]
    y, msg, it = kkt(lsq, H, beta, terms, y0)
    assert msg == 6 and it == 0 and np.array_equal(y, y0)
    res = np.zeros(k + 1)
    res[0] = beta

    def func(v):
        return float(np.sum((res - H @ v) ** 2))

    def jac(v):
        return -2 * H.T @ (res - H @ v)

    cl = [{"type": "eq", "fun": (lambda v, a=a, b=b, c=c: a + b @ v + v @ c @ v),
           "jac": (lambda v, b=b, c=c: b + 2 * (v @ c))} for a, b, c in terms]
    sol = _slsqp(func, y0, jac, cl, 1e-24)
    assert sol.message == "Singular matrix C in LSQ subproblem"
    np.testing.assert_array_equal(sol.x, y)
    assert max(f["fun"](y) for f in cl) > 1e-12  # the reference's checker then falls back


@pytest.mark.parametrize("case", ["kkt_c5_cycle8", "kkt_c5_cycle9", "kkt_c5_onereduce_cycle0"])
def test_kkt_c5_restart_cycles_match_slsqp(lsq, case):
    """Config C5's forced constrained steps (swe M=913, mass + energy + the synthetic third
    constraint, restarted CGMRES(30)) as the round-2 device solver received them (H, beta, warm
    start and the three reduced constraints, tools/dump_c5_kkt.py): x0 already satisfies every
    constraint (term0 = 0) and the mass constraint's gradient is roundoff (|term1| ~ 1e-12).  On
    these inputs the reference's SLSQP (solvers.py:251-255) returns a feasible point (at its
    iteration limit for cycle 8, so the branch is "con" with a RuntimeWarning; cycle 0 of the
    round-3 one-reduce MGS as well), while Newton on
    ||F|| from both of its starts converged to a constrained saddle (cycle 8: f = 2.3e-2 against
    SLSQP's 7.0e-3) and the device fell back.  The SQP solve must find SLSQP's minimum."""
    import os
    from oracle.cgmres_port import _slsqp

    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "kkt_cases", case + ".npz"))
    H, beta, y0 = z["H"], float(z["beta"]), z["y0"]
    k = H.shape[1]
    terms = [(z["t0"][i], z["t1"][i], z["t2"][i]) for i in range(len(z["t0"]))]
    res = np.zeros(k + 1)
    res[0] = beta

    def func(v):
        return float(np.sum((res - H @ v) ** 2))

    def jac(v):
        return -2 * H.T @ (res - H @ v)

    cl = [{"type": "eq", "fun": (lambda v, a=a, b=b, c=c: a + b @ v + v @ c @ v),
           "jac": (lambda v, b=b, c=c: b + 2 * (v @ c))} for a, b, c in terms]
    sol = _slsqp(func, y0, jac, cl, 1e-24)
    assert max(f["fun"](sol.x) for f in cl) <= 1e-12  # the reference keeps its constrained step
    y, msg, _ = kkt(lsq, H, beta, terms, y0)
    assert msg == 0
    for t0, t1, t2 in terms:  # the signed checker passes (solvers.py:267)
        assert lsq.lsq_con_value(k, t0, _p(t1), _p(t2), _p(y)) <= 1e-12
    # each constraint ends 8 eps x its rounding scale on the feasible side (so that the signed
    # checker passes on the computed value), which may cost up to sum |lambda_i| 16 eps scale_i
    # (kkt_c5_onereduce_cycle0, the one-reduce MGS's inputs of cycle 0: the third constraint's
    # scale is 6e7, its margin 1e-7, the objective 2e-10 relative above SLSQP's)
    eps = np.finfo(float).eps
    G = np.stack([b + 2 * (y @ c) for _, b, c in terms], 1)
    lam = np.linalg.lstsq(G, -jac(y), rcond=None)[0]
    scale = [abs(a) + np.abs(b) @ np.abs(y) + np.abs(y) @ np.abs(c) @ np.abs(y) for a, b, c in terms]
    margin = sum(abs(li) * 16 * eps * si for li, si in zip(lam, scale))
    assert func(y) <= func(sol.x) * (1 + 1e-12) + margin
    assert np.linalg.norm(y - sol.x) <= 1e-6 * np.linalg.norm(sol.x)


def test_kkt_checker_sign_at_rounding_floor(lsq):
    """swe M=30 CGMRES(25)'s forced constrained step as the device solver received it (SpMV mode
    "off", tools/dump_pipe_modes_kkt.py): the warm start already sits at the rounding floor
    (f ~ 1e-21), with the mass constraint's value +1.8e-12 as the reference's checker evaluates
    it.  The solve must not stop there: the constraint values it tests are the unscaled ones, the
    checker's (solvers.py:14-18,267), so the returned y passes the signed check."""
    import os

    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "kkt_cases", "kkt_swe_m30_final_step.npz"))
    H, beta, y0 = z["H"], float(z["beta"]), z["y0"]
    k = H.shape[1]
    terms = [(z["t0"][i], z["t1"][i], z["t2"][i]) for i in range(len(z["t0"]))]
    assert max(lsq.lsq_con_value(k, a, _p(b), _p(c), _p(y0)) for a, b, c in terms) > 1e-12
    y, msg, _ = kkt(lsq, H, beta, terms, y0)
    assert msg == 0
    for t0, t1, t2 in terms:
        assert lsq.lsq_con_value(k, t0, _p(t1), _p(t2), _p(y)) <= 0.0
    res = np.zeros(k + 1)
    res[0] = beta
    assert np.sum((res - H @ y) ** 2) <= 1e-20 * beta ** 2


@pytest.mark.parametrize("case", ["kkt_c5_cycle8", "kkt_swe_m30_final_step"])
def test_kkt_initial_multipliers_on_scaled_jacobian(lsq, case):
    """the SQP's starting multipliers are the least-squares fit
    (J_s J_s') lam = -J_s grad f on the constraint Jacobian scaled to unit rows at y0, the same
    scaled constraints the SQP iterates on.  Round 3 formed J from the unscaled term1 plus the
    scaled term2 (neither Jacobian), which brought back the ~1e9 mass multiplier the scaling
    removes (C5 cycle 8: |term1| ~ 1e-11)."""
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "kkt_cases", case + ".npz"))
    H, beta, y0 = z["H"], float(z["beta"]), z["y0"]
    t0, t1, t2 = z["t0"], z["t1"], z["t2"]
    p, m = H.shape[1], len(t0)
    L = lsq
    L.lsq_kkt_init_multipliers.argtypes = [C.c_int, PD, C.c_double, C.c_int, PD, PD, PD, PD, PD]
    lam = np.zeros(m)
    Hc = np.asfortranarray(H)
    assert L.lsq_kkt_init_multipliers(p, Hc.ctypes.data_as(PD), beta, m, _p(t0), _p(t1.ravel()), _p(t2.ravel()),
                                      _p(y0), lam.ctypes.data_as(PD)) == 0
    rhs = np.zeros(p + 1)
    rhs[0] = beta
    grad = -2 * H.T @ (rhs - H @ y0)
    J = np.stack([t1[i] + (t2[i] + t2[i].T) @ y0 for i in range(m)])
    Js = J / np.linalg.norm(J, axis=1)[:, None]
    ref = np.linalg.solve(Js @ Js.T, -Js @ grad)
    # grad f is formed from R, g on the host side and from H here: equal to its terms' rounding
    gscale = 2 * (np.abs(H.T) @ (np.abs(H) @ np.abs(y0) + np.abs(rhs))).max()
    np.testing.assert_allclose(lam, ref, rtol=1e-8, atol=1e-12 * gscale)
    # unit-gradient constraints: multipliers of the objective's own scale, not the 1e9 of round 3
    assert np.abs(lam).max() <= 10 * np.linalg.norm(grad)
