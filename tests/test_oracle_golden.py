"""Pin the oracle (CPU restatement, ``oracle/cgmres_port.py``) to the golden
vectors produced by the reference ``solvers.py`` itself
(``tests/golden/make_golden.py``).  Same NumPy/SciPy primitives in the same
order => the results must be identical to the last bit."""
import warnings

import numpy as np
import pytest

import oracle
from _golden import Case, expected_trace, names


def _run_oracle(case, trace):
    kw = case.kwargs()
    pre = case.preconditioner()
    if case.solver == "gmres":
        return oracle.gmres(case.A, case.b, case.x0, case.k, tol=case.tol, pre=pre)
    if case.solver == "cgmres_p":
        return oracle.cgmres_p(case.A, case.b, case.x0, case.k, conlist=case.conlist(), pre=pre, trace=trace)
    return oracle.cgmres(case.A, case.b, case.x0, case.k, tol=case.tol, conlist=case.conlist(), pre=pre,
                         trace=trace, **kw)


@pytest.mark.parametrize("name", names())
def test_oracle_matches_reference_bitwise(name):
    case = Case(name)
    trace = []
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        x, d = _run_oracle(case, trace)
    timing = bool(case.meta.get("timing"))
    if not timing:
        np.testing.assert_array_equal(np.asarray(d["x"]), case.x_all)
        np.testing.assert_array_equal(x, case.x_final)
        np.testing.assert_array_equal(np.asarray(d["res"]), case.res)
    else:  # timing=True skips the NaN/checker paths but must produce the same iterates
        np.testing.assert_array_equal(np.asarray(d["x"]), case.x_all)
        assert sorted(d["timings"].keys()) == [str(k) for k in case.z["timing_keys"]]
        assert d["timings"]["constrained_steps"] == int(case.z["timing_constrained_steps"])
    if "steps" in d:
        assert d["steps"] == case.steps
    assert [str(w.message) for w in caught] == case.py_warnings
    if case.solver != "gmres":
        assert trace == expected_trace(case)
