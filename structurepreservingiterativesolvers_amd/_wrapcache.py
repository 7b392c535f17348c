"""Cache of operators the wrappers derive from the problem dict on every call
(``M + 0.5*dt*L`` in ``heat/LinearSolver.py:33``, ``L - M`` in
``lkdv/LinearSolver.py:42``, lifted lkdvRK operators).  The reference rebuilds
them per call; here they are built once per (source objects, parameters) so
that the HBM upload cache (keyed on object identity) stays warm across calls
with the same problem dict."""
from __future__ import annotations

import weakref

import numpy as np

_CACHE: dict = {}


def derived(sources, params, build):
    key = tuple(id(s) for s in sources) + tuple(params)
    hit = _CACHE.get(key)
    if hit is not None:
        return hit
    val = build()
    _CACHE[key] = val
    for s in sources:
        try:
            weakref.finalize(s, _CACHE.pop, key, None)
        except TypeError:
            pass
    return val


_ZEROS: dict = {}


def zeros(n):
    """A read-only all-zero fp64 vector of length ``n``, shared: the wrappers' ``np.zeros_like(x0)``
    constraint vectors (``swe/LinearSolver.py:36``, ``lkdv/LinearSolver.py``), made once instead of
    an 8 MB allocation per call; the solver skips its zero test (:func:`is_known_zero`)."""
    n = int(n)
    z = _ZEROS.get(n)
    if z is None:
        if len(_ZEROS) >= 4:
            _ZEROS.pop(next(iter(_ZEROS)))
        z = np.zeros(n)
        z.setflags(write=False)
        _ZEROS[n] = z
    return z


def is_known_zero(v):
    """``v`` is one of :func:`zeros`'s shared read-only vectors (read-only: never edited since)."""
    return type(v) is np.ndarray and _ZEROS.get(v.size) is v
