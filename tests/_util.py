"""Shared helpers of the test-suite."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# fp64 tolerance of the HIP solve vs the oracle: |d| <= TOL * max(1, |ref|)
# with an identical decision trace.  The model arithmetic differs from CasADi's QR at
# ~1e-11 relative (tests/test_model_host.py), which the solve amplifies to <~1e-8.
SOLVE_TOL = 1e-6
# per-function tolerance of the hand-written model vs the CasADi kernels.  Measured worst
# cases over the 64 KAT states (host build, tests/test_model_host.py): values 1.5e-10
# (Dyn_FL, Imp_B), Jacobians 1.4e-9 (Dyn_FL_par); CasADi's QR leaves ~1e-10 noise itself.
KAT_TOL = {"value": 1e-9, "jac": 5e-9}


def golden(name):
    return dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))


def rel_err(a, b):
    a = np.asarray(a, dtype=float)
    b = np.asarray(b, dtype=float)
    if a.size == 0:
        return 0.0
    return float(np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b))))
