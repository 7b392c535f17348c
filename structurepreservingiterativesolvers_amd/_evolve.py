"""Time-stepping driver shared by the per-problem ``Evolve`` modules (the outer loop of
``lkdv/Evolve.py:19-64``, ``swe/Evolve.py:18-56``, ``lkdvRK/Evolve.py:19-92``).

The reference rebuilds every form with ``linforms(..., zinit=sol[-1])`` each step, so its
operators are fresh objects per step.  Here ``step_forms`` keeps ``A``/``M``/``L``/``omega``
(and the matrices derived from them) as the same objects, so the HBM upload cache hits on every
step and a step costs one rhs/target update on the host plus the solve on the device.  Each
step's device Krylov basis is released once its state has been read back."""
from __future__ import annotations

import numpy as np


def _release(d):
    x = d.get("x") if isinstance(d, dict) else None
    if x is not None and hasattr(x, "release"):
        x.release()


def run(forms, prob, n_solves, step_forms, solve, state, invariants, names, dt_out, extra=None):
    """Advance ``n_solves`` steps.

    ``solve(forms, x_prev) -> (x, dict)``; ``state(forms, x) -> z`` maps the solver's unknown to
    the new state; ``invariants(forms, x) -> dict`` with keys ``names``; ``extra(forms, x, t)``
    returns an extra per-step scalar (lkdvRK's error) or None.  Returns the reference's ``out``
    dict with numpy states in ``sol`` (the reference stores Firedrake functions)."""
    sol = [np.asarray(forms["z0"], dtype=np.float64).copy()]
    time = [0.0]
    hist = {nm: [float(forms[key])] for nm, key in names}
    err = [0.0]
    x = None
    for i in range(1, n_solves + 1):
        forms = step_forms(forms, sol[-1])
        x, d = solve(forms, x)
        x = np.asarray(x, dtype=np.float64)
        _release(d)
        inv = invariants(forms, x)
        for nm, _ in names:
            hist[nm].append(inv[nm])
        sol.append(state(forms, x))
        time.append(dt_out * i)
        if extra is not None:
            err.append(extra(forms, x, time[-1]))
    out = {"sol": sol, "time": time}
    if extra is not None:
        out["err"] = err
    short = {"mass": "dm", "momentum": "dmo", "energy": "de"}
    for nm, _ in names:
        h = np.asarray(hist[nm])
        out[short[nm]] = np.abs(h - h[0])
    return out
