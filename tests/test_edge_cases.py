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


def test_overflow_case_conditioning():
    """Why the overflow case is held to 1e-3 and not the solve tests' 1e-6
    (tests/test_gpu_edge_cases.py): the oracle itself, given x0 perturbed by 1e-13 relative
    (far below the device model's ~1e-11 difference to the reference's CasADi kernels),
    takes the same decisions but moves its finite outputs by more than 1e-4 -- the surviving
    violent trajectories amplify input rounding ~1e9..1e10, so no implementation that rounds
    differently can meet 1e-6 there.  The armijo case, for contrast, moves by < 1e-7."""
    if not O.available():
        pytest.skip("oracle not built")

    def spread(name, eps=1e-13):
        desc, opt, x0 = E.inputs(name, batch=32)
        ref = O.solve(desc, opt.to_c(), x0, nthreads=8)
        rng = np.random.default_rng(1)
        got = O.solve(desc, opt.to_c(), x0 * (1 + eps * rng.standard_normal(x0.shape)), nthreads=8)
        assert (got["trace"] == ref["trace"]).all() and (got["status"] == ref["status"]).all()
        e = 0.0
        for k in ("X", "U", "K", "DU", "G"):
            a, b = np.asarray(got[k], float), np.asarray(ref[k], float)
            f = np.isfinite(a) & np.isfinite(b)
            e = max(e, float(np.max(np.abs(a[f] - b[f]) / np.maximum(1.0, np.abs(b[f])))))
        return e

    e_over, e_armijo = spread("nonfinite"), spread("armijo_a")
    print(f"oracle spread under a 1e-13 x0 perturbation: overflow case {e_over:.1e}, "
          f"armijo case {e_armijo:.1e}")
    assert e_over > 1e-4
    assert e_armijo < 1e-7
