"""Drop-in for the reference ``swe/Evolve.py:18-56``: linear rotating shallow water over
``N - 1`` steps from ``x0 = 0`` (``:43``); mass and energy deviations.  The reference returns
from inside its loop (``:51-55``, so ``N = 1`` has no ``out``); here ``N = 1`` returns the
initial state only."""
import numpy as np

from .. import _evolve
from . import LinearSolver as ls
from . import assembly as asm


def evolve(N=100, M=50, degree=1, k=50, tol=1e-6, solver=ls.cgmresWrapper):
    forms, prob = asm.linforms(N=N, M=M, degree=degree)
    return _evolve.run(
        forms, prob, N - 1, asm.step_forms,
        solve=lambda f, x: solver(f, x0=np.zeros_like(f["b"]), k=k, tol=tol),
        state=lambda f, x: x.copy(),
        invariants=lambda f, x: asm.compute_invariants(prob, f, x),
        names=[("mass", "m0"), ("energy", "e0")],
        dt_out=forms["T"] / N,
    )
