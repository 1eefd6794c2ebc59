"""The backward sweep's PSD verdict on Quu - 1e-9 I (SinglePhase.cpp:202-209,
Eigen::LDLT::isPositive): the kernel (mhpc_bws.hip, MHPC_BWS_PSD=1) runs an unpivoted LDL^T
instead of Eigen's diagonally pivoted one.  Both are restated here in numpy -- the pivoted
one exactly as oracle/hsddp_oracle.cpp restates Eigen's ldlt_inplace<Lower>::unblocked --
and must give the same verdict on positive-definite, indefinite, rank-deficient and
near-singular (smallest |eigenvalue| 1e-12..1e-6) symmetric 4x4 matrices wherever the
verdict is decided by the matrix and not by rounding: |smallest eigenvalue| above
1e-10 x the largest entry.  Inside that band the verdict is round-off noise for either
algorithm (the GPU's Quu already differs from the oracle's in the last bits), and the two
are only reported.""" 
import numpy as np
import pytest


def pivoted_is_positive(A):
    A = A.copy()
    out = np.zeros(len(A), dtype=bool)
    for b in range(len(A)):
        M = A[b]
        sign, stop = 0, False  # 0 ZeroSign, 1 PositiveSemiDef, 2 NegativeSemiDef, 3 Indefinite
        for k in range(4):
            big = k + int(np.argmax(np.abs(np.diag(M)[k:])))
            if big != k:  # symmetric transposition
                M[[k, big]] = M[[big, k]]
                M[:, [k, big]] = M[:, [big, k]]
            if k > 0:
                temp = np.array([M[j, j] * M[k, j] for j in range(k)])
                M[k, k] -= sum(M[k, j] * temp[j] for j in range(k))
                for i in range(k + 1, 4):
                    M[i, k] -= sum(M[i, j] * temp[j] for j in range(k))
            akk = M[k, k]
            valid = abs(akk) > 0
            if k == 0:
                stop = not valid
            if valid:
                for i in range(k + 1, 4):
                    M[i, k] /= akk
            ns = sign
            if sign == 1:
                ns = 3 if akk < 0 else 1
            elif sign == 2:
                ns = 3 if akk > 0 else 2
            elif sign == 0:
                ns = 1 if akk > 0 else (2 if akk < 0 else 0)
            sign = 0 if stop else ns
        out[b] = sign in (0, 1)
    return out


def unpivoted_is_positive(A):
    """mhpc_bws.hip:ldlt_nopiv_is_positive4, vectorised over matrices."""
    A = A.copy()
    neg = np.zeros(len(A), dtype=bool)
    for k in range(4):
        akk = A[:, k, k].copy()
        neg |= akk < 0
        valid = akk != 0
        r = 1.0 / np.where(valid, akk, 1.0)
        for i in range(k + 1, 4):
            li = A[:, i, k] * r
            for j in range(k + 1, i + 1):
                A[:, i, j] -= np.where(valid, li * A[:, j, k], 0.0)
                A[:, j, i] = A[:, i, j]
    return ~neg


@pytest.mark.parametrize("kind", ["pd", "indefinite", "rank_deficient", "near_singular"])
def test_unpivoted_verdict_matches_pivoted(kind):
    rng = np.random.default_rng(7)
    n = 1500
    X = rng.standard_normal((n, 4, 4)) * 10 ** rng.uniform(-3, 3, (n, 1, 1))
    if kind == "pd":
        A = X @ X.transpose(0, 2, 1) + 1e-3 * np.eye(4)
    elif kind == "indefinite":
        A = X + X.transpose(0, 2, 1)
    elif kind == "rank_deficient":
        Y = X[:, :, :3]
        A = Y @ Y.transpose(0, 2, 1)
    else:
        Q, _ = np.linalg.qr(rng.standard_normal((n, 4, 4)))
        ev = 10 ** rng.uniform(-2, 3, (n, 4))
        ev[:, 0] = rng.choice([-1.0, 1.0], n) * 10 ** rng.uniform(-12, -6, n)
        A = Q @ (ev[:, :, None] * Q.transpose(0, 2, 1))
    A = 0.5 * (A + A.transpose(0, 2, 1)) - 1e-9 * np.eye(4)
    a, b = pivoted_is_positive(A), unpivoted_is_positive(A)
    lam = np.abs(np.linalg.eigvalsh(A)).min(axis=1)
    decided = lam > 1e-10 * np.abs(A).max(axis=(1, 2))
    print(f"{kind}: {int(decided.sum())} decided, disagreements {int((a != b)[decided].sum())}; "
          f"in the round-off band {int((~decided).sum())}, disagreements {int((a != b)[~decided].sum())}")
    assert decided.sum() > n // 3
    assert (a == b)[decided].all()
    if kind == "pd":
        assert a.all()
    if kind == "indefinite":
        assert a.mean() < 0.05
