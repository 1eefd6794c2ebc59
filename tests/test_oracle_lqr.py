"""The oracle's Riccati step against an independent dense solve (CPU only).

oracle_riccati_knot runs one knot of SinglePhase::backward_sweep exactly as the oracle does
(compute_Qfunction + regularisation, the PSD test, valuefunction_update;
MHPC_CompoundTypes.h:117-144, SinglePhase.cpp:197-212).  Here the same stage is solved
without any of those formulas: for a fixed state x, minimise the stage cost plus the next
value function over (u, y, x') subject to the dynamics x' = A x + B u and the outputs
y = C x + D u, by one dense KKT system (numpy.linalg.solve).  The optimal control is affine
in x (du = u*(0), K e_i = u*(e_i) - u*(0)) and the optimal value V(x) quadratic, so G and H
follow from V at 0, +-e_i, e_i + e_j.  The oracle must agree to round-off, and its dV must be
-Qu' Quu^-1 Qu = 2 V(0) (quirk B3: no 1/2).  Its LDL^T PSD verdict must agree with the
eigenvalue signs of symmetric matrices whose spectrum stays clear of zero."""
import ctypes

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.skipif(not O.available(), reason="oracle not built")


def _p(a):
    return np.ascontiguousarray(a, dtype=np.float64).ctypes.data_as(ctypes.c_void_p)


def oracle_knot(n, blk, reg):
    L = O.lib()
    L.oracle_riccati_knot.restype = ctypes.c_int
    K, du, G, H, dV = np.zeros((4, n)), np.zeros(4), np.zeros(n), np.zeros((n, n)), ctypes.c_double()
    keep = [np.ascontiguousarray(blk[k], dtype=np.float64) for k in
            ("A", "B", "C", "D", "lx", "lu", "ly", "lxx", "lux", "luu", "lyy", "G", "H")]
    ok = L.oracle_riccati_knot(ctypes.c_int(n), *[k.ctypes.data_as(ctypes.c_void_p) for k in keep],
                               ctypes.c_double(reg), _p(K), _p(du), _p(G), _p(H), ctypes.byref(dV))
    # outputs were written through fresh arrays: _p() returns pointers into them directly
    return ok, K, du, G, H, dV.value


def random_stage(rng, n, stance):
    A = np.eye(n) + 0.01 * rng.standard_normal((n, n))
    B = 0.1 * rng.standard_normal((n, 4))
    C = rng.standard_normal((4, n)) if stance else np.zeros((4, n))
    D = rng.standard_normal((4, 4)) if stance else np.zeros((4, 4))
    S = rng.standard_normal((n, n))
    H = S @ S.T + np.eye(n)
    Y = rng.standard_normal((4, 4))
    return {
        "A": A, "B": B, "C": C, "D": D,
        "lx": rng.standard_normal(n), "lu": rng.standard_normal(4), "ly": rng.standard_normal(4),
        "lxx": np.diag(rng.uniform(0.01, 1.0, n)), "lux": 0.1 * rng.standard_normal((4, n)),
        "luu": np.diag(rng.uniform(0.1, 1.0, 4)), "lyy": Y @ Y.T if stance else np.zeros((4, 4)),
        "G": rng.standard_normal(n), "H": H,
    }


def kkt_value(blk, reg, x):
    """min over (u, y, x') of the stage cost + next value at state x; returns (u*, V)."""
    n = len(x)
    W = np.zeros((8 + n, 8 + n))
    W[:4, :4] = blk["luu"] + reg * np.eye(4)
    W[4:8, 4:8] = blk["lyy"]
    W[8:, 8:] = blk["H"]
    w = np.concatenate([blk["lu"] + blk["lux"] @ x, blk["ly"], blk["G"]])
    E = np.zeros((4 + n, 8 + n))
    E[:4, :4] = -blk["D"]
    E[:4, 4:8] = np.eye(4)
    E[4:, :4] = -blk["B"]
    E[4:, 8:] = np.eye(n)
    e = np.concatenate([blk["C"] @ x, blk["A"] @ x])
    M = np.block([[W, E.T], [E, np.zeros((4 + n, 4 + n))]])
    sol = np.linalg.solve(M, np.concatenate([-w, e]))
    v = sol[:8 + n]
    V = blk["lx"] @ x + 0.5 * x @ (blk["lxx"] + reg * np.eye(n)) @ x + 0.5 * v @ W @ v + w @ v
    return v[:4], V


@pytest.mark.parametrize("n,stance,reg", [(14, True, 0.0), (14, False, 0.0), (14, True, 1e-3),
                                          (6, False, 0.0), (6, False, 0.5)])
def test_riccati_knot_is_the_exact_lq_solution(n, stance, reg):
    rng = np.random.default_rng(1000 * n + 10 * stance + int(reg * 1e3))
    for _ in range(20):
        blk = random_stage(rng, n, stance)
        ok, K, du, G, H, dV = oracle_knot(n, blk, reg)
        assert ok == 1
        u0, V0 = kkt_value(blk, reg, np.zeros(n))
        I = np.eye(n)
        Kx = np.stack([kkt_value(blk, reg, I[i])[0] - u0 for i in range(n)], axis=1)
        Vp = np.array([kkt_value(blk, reg, I[i])[1] for i in range(n)])
        Vm = np.array([kkt_value(blk, reg, -I[i])[1] for i in range(n)])
        Gx = (Vp - Vm) / 2
        Hx = np.array([[kkt_value(blk, reg, I[i] + I[j])[1] - Vp[i] - Vp[j] + V0
                        for j in range(n)] for i in range(n)])
        scale = lambda a: max(1.0, float(np.max(np.abs(a))))  # noqa: E731
        assert np.max(np.abs(du - u0)) <= 1e-10 * scale(u0)
        assert np.max(np.abs(K - Kx)) <= 1e-10 * scale(Kx)
        assert np.max(np.abs(G - Gx)) <= 1e-9 * scale(Gx)
        assert np.max(np.abs(H - Hx)) <= 1e-9 * scale(Hx)
        # quirk B3: dV = -Qu' Quu^-1 Qu, twice the exact optimal decrease V(0) - 0
        assert abs(dV - 2 * V0) <= 1e-10 * max(1.0, abs(V0))


def test_riccati_knot_rejects_an_indefinite_quu():
    rng = np.random.default_rng(7)
    blk = random_stage(rng, 14, False)
    blk["luu"] = np.diag([1.0, 1.0, -50.0, 1.0])  # Quu = luu + B'HB with B small: indefinite
    ok = oracle_knot(14, blk, 0.0)[0]
    assert ok == 0
    assert oracle_knot(14, blk, 100.0)[0] == 1  # the regularisation retry makes it PD


def test_ldlt_verdict_matches_eigenvalue_signs():
    L = O.lib()
    L.oracle_ldlt_is_positive.restype = ctypes.c_int
    rng = np.random.default_rng(11)
    agree = 0
    for t in range(2000):
        Q, _ = np.linalg.qr(rng.standard_normal((4, 4)))
        mag = 10.0 ** rng.uniform(-6, 2, 4)
        sgn = np.where(rng.random(4) < (0.8 if t % 2 else 0.2), 1.0, -1.0)
        A = (Q * (sgn * mag)) @ Q.T
        A = (A + A.T) / 2
        lam = np.linalg.eigvalsh(A)
        if np.min(np.abs(lam)) < 1e-9 * np.max(np.abs(lam)):
            continue  # verdict decided by rounding, not by the matrix
        got = L.oracle_ldlt_is_positive(_p(A)) == 1
        assert got == bool(lam.min() > 0), (A, lam)
        agree += 1
    assert agree > 1900
