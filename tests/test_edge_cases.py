"""The rarely taken branches of MultiPhaseDDP::solve (tests/_edge_cases.py): the CPU oracle
against its committed fixtures, and the fixtures against the branches they must reach.

GPU parity for the same inputs: tests/test_gpu_edge_cases.py."""
import numpy as np
import pytest

import _edge_cases as E
from _util import golden

import oracle as O

need_oracle = pytest.mark.skipif(not O.available(), reason="oracle not built")


def test_fixtures_reach_the_branches():
    g = golden("edge_reg_abort.npz")
    # quirk B8: the abort trace entry (bit 21) and the status, for some but not all problems
    aborted = ((g["trace"] > 0) & ((g["trace"] >> 21) & 1 == 1)).any(axis=1)
    assert 0 < aborted.sum() < len(aborted)
    np.testing.assert_array_equal(g["status"] == 1, aborted)
    # Armijo: first acceptance at every trial j = 2..9 of the 29-trial grid, plus none (30)
    seen = set(E.n_ls(golden("edge_armijo_a.npz")["trace"]).tolist()) | \
        set(E.n_ls(golden("edge_armijo_b.npz")["trace"]).tolist())
    assert set(range(1, 10)) <= seen and 30 in seen, sorted(seen)
    g = golden("edge_nonfinite.npz")
    bad = ~np.isfinite(g["J"])
    assert 0 < bad.sum() < len(bad)
    np.testing.assert_array_equal(g["status"] == 2, bad)


@need_oracle
@pytest.mark.parametrize("name", sorted(E.CASES))
def test_oracle_reproduces_edge_fixture(name):
    desc, opt, x0 = E.inputs(name)
    g = golden(f"edge_{name}.npz")
    np.testing.assert_array_equal(g["x0"], x0)
    r = O.solve(desc, opt.to_c(), x0, nthreads=8)
    for k in ("trace", "status", "counters"):
        np.testing.assert_array_equal(r[k], g[k], err_msg=k)
    for k in ("J", "dV_exp", "viol", "V", "dV"):
        np.testing.assert_array_equal(r[k], g[k], err_msg=k)
