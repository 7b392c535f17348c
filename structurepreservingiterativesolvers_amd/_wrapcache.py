"""Cache of operators the wrappers derive from the problem dict on every call
(``M + 0.5*dt*L`` in ``heat/LinearSolver.py:33``, ``L - M`` in
``lkdv/LinearSolver.py:42``, lifted lkdvRK operators).  The reference rebuilds
them per call; here they are built once per (source objects, parameters) so
that the HBM upload cache (keyed on object identity) stays warm across calls
with the same problem dict."""
from __future__ import annotations

import weakref

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
