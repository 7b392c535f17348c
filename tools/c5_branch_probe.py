"""C5-shaped branch probe on the CPU: restarted CGMRES(k) on swe M with the synthetic third
constraint (bench.py --config c5), run through the ORACLE (the reference's arithmetic, SLSQP).
At every cycle's constrained step the host KKT (liblsq_host.so) is run on the oracle's own
inputs (H, beta, warm start, reduced terms) and the two outcomes are compared:

    python tools/c5_branch_probe.py [M] [cycles] [k]

Prints one line per cycle: the oracle's branch sequence tail, SLSQP's message and max
constraint value, the KKT message / max constraint value, and |y_kkt - y_slsqp|."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle.cgmres_port import ConstraintTerms, _Arnoldi, _slsqp  # noqa: E402
from structurepreservingiterativesolvers_amd.swe import LinearSolver as ls  # noqa: E402
from structurepreservingiterativesolvers_amd.swe import assembly  # noqa: E402


def _kkt_lib():
    import ctypes as C

    PD = C.POINTER(C.c_double)
    L = C.CDLL(os.path.join(ROOT, "structurepreservingiterativesolvers_amd", "liblsq_host.so"))
    L.lsq_kkt_solve.argtypes = [C.c_int, PD, C.c_double, C.c_int, PD, PD, PD, PD, PD, C.POINTER(C.c_int),
                                C.POINTER(C.c_int)]
    L.lsq_con_value.argtypes = [C.c_int, C.c_double, PD, PD, PD]
    L.lsq_con_value.restype = C.c_double
    return L


def kkt(L, Hj, beta, terms, y0):
    import ctypes as C

    PD = C.POINTER(C.c_double)

    def p_(a):
        return np.ascontiguousarray(a, dtype=np.float64).ctypes.data_as(PD)

    p = Hj.shape[1]
    t0 = np.array([t[0] for t in terms])
    t1 = np.concatenate([t[1] for t in terms])
    t2 = np.concatenate([np.ascontiguousarray(t[2]).ravel() for t in terms])
    y = np.zeros(p)
    msg, it = C.c_int(), C.c_int()
    Hc = np.asfortranarray(Hj)
    L.lsq_kkt_solve(p, Hc.ctypes.data_as(PD), beta, len(terms), p_(t0), p_(t1), p_(t2), p_(y0),
                    y.ctypes.data_as(PD), C.byref(msg), C.byref(it))
    cv = [L.lsq_con_value(p, t[0], p_(t[1]), p_(t[2]), p_(y)) for t in terms]
    return y, msg.value, it.value, cv


def cycle(A, b, x0, k, cons, L, dump=None):
    """One reference cgmres call (tol=1e-19: k-1 unconstrained steps + the forced constrained
    one), restated step by step so the constrained step's inputs can be handed to the KKT."""
    st = _Arnoldi(A, b, x0, k, None)
    yk = None
    for j in range(k):
        st.extend(j)
        _, func, jac = st.ls_objective(j)
        y0 = np.zeros(j + 1)
        if j:
            y0[:-1] = yk
        if j < k - 1:
            yk = _slsqp(func, y0, jac, [], 1e-24).x
    Z = st.basis(k - 1)
    terms = [ConstraintTerms(c, x0, Z) for c in cons]
    eq = [t.as_slsqp() for t in terms]
    sol = _slsqp(func, y0, jac, eq, 1e-24)
    cvs = max(0, *[e["fun"](sol.x) for e in eq])
    branch = "con" if not np.isnan(sol.x).any() and cvs <= 1e-12 else "fallback"
    tt = [(t.term0, t.term1, t.term2) for t in terms]
    y, msg, it, cv = kkt(L, st.H[: k + 1, :k], st.beta, tt, y0)
    kb = "con" if msg in (0,) or (max(0, *cv) <= 1e-12 and msg != 6) else "fallback"
    if dump:
        np.savez(dump, H=st.H[: k + 1, :k], beta=st.beta, y0=y0, t0=np.array([t[0] for t in tt]),
                 t1=np.stack([t[1] for t in tt]), t2=np.stack([t[2] for t in tt]), y_slsqp=sol.x,
                 msg_slsqp=str(sol.message), nit_slsqp=sol.nit)
    if branch == "con":
        x = Z @ sol.x + x0
    else:
        x = Z @ _slsqp(func, y0, jac, [], 1e-24).x + x0
    return x, dict(branch=branch, msg=sol.message, nit=sol.nit, cv_slsqp=cvs, kkt_msg=msg, kkt_it=it,
                   cv_kkt=max(cv), kkt_branch=kb, dy=float(np.abs(y - sol.x).max()),
                   f_slsqp=func(sol.x), f_kkt=func(y), res=np.linalg.norm(A @ x - b))


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    cycles = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    dump_dir = sys.argv[4] if len(sys.argv) > 4 else None
    dic, _ = assembly.linforms(M=M)
    n = dic["A"].shape[0]
    x = np.zeros(n)
    cons = ls.constraints(dic, x)
    D, c3 = assembly.extra_constraint(n, dic["z0"], seed=2)
    cons.append(ls._Constraint(D, np.zeros(n), c3))
    L = _kkt_lib()
    for c in range(cycles):
        t = time.time()
        dump = os.path.join(dump_dir, f"kkt_c5probe_M{M}_cycle{c}.npz") if dump_dir else None
        x, r = cycle(dic["A"], dic["b"], x, k, cons, L, dump)
        print(f"M={M} cycle {c}: ref {r['branch']:8s} slsqp '{r['msg']}' nit={r['nit']} cv={r['cv_slsqp']:.2e} | "
              f"kkt {r['kkt_branch']:8s} msg={r['kkt_msg']} it={r['kkt_it']} cv={r['cv_kkt']:.2e} | "
              f"dy={r['dy']:.2e} f {r['f_slsqp']:.6e} vs {r['f_kkt']:.6e} res={r['res']:.3e} ({time.time() - t:.1f}s)",
              flush=True)


if __name__ == "__main__":
    main()
