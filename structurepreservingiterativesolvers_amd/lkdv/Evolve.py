"""Drop-in for the reference ``lkdv/Evolve.py:19-64``: implicit-midpoint linear KdV over
``N - 1`` steps, each solved from ``x0 = 0`` (``:45``).  ``sol`` holds numpy states; the
reference appends one Firedrake function object repeatedly (``:49-55``), so its list aliases
the last state, while here every entry is that step's state."""
import numpy as np

from .. import _evolve
from . import LinearSolver as ls
from . import assembly as asm


def evolve(N=100, M=50, degree=1, k=50, tol=1e-6, contol=10, solver=ls.cgmresWrapper):
    forms, prob = asm.linforms(N=N, M=M, degree=degree)
    return _evolve.run(
        forms, prob, N - 1, asm.step_forms,
        solve=lambda f, x: solver(f, x0=np.zeros_like(f["b"]), k=k, tol=tol, contol=contol),
        state=lambda f, x: x.copy(),
        invariants=lambda f, x: asm.compute_invariants(prob, f, x),
        names=[("mass", "m0"), ("momentum", "mo0"), ("energy", "e0")],
        dt_out=forms["T"] / N,
    )
