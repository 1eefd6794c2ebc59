"""C5 in the fp32 instantiation (BASELINE.json configs[4], SURVEY.md 8c: "fp32 (C5) is
compared to the fp64 oracle with the trace-divergence rate reported").  fp32 cannot follow
the fp64 decision trace bit for bit (a line-search acceptance or a PSD test near its
threshold flips under fp32 round-off), so the test reports the divergence rate and bounds
it, and bounds the cost error of the problems that took the same decisions."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# Measured on MI355X (round 3): 64 problems -- traces identical 64/64, relative cost error
# median 1.4e-5, max 1.8e-3; the batch-4103 sample of test_gpu_variants.py -- traces 63/63
# (distinct indices), max 1.4e-3.  The fp32 build sums costs and compares the Armijo
# condition in fp64 (mhpc_solver.h `acc`) and inverts the whole-body knots' 4x4 control block
# in fp64 (mhpc_bws.hip, MHPC_BWS_WIDE): the gains of one fp32 sweep were 1e-2 off in the
# stance phases (tools/diag_fp32_stages.py), the source of the earlier 5e-3..1e-2 cost errors;
# fp64 cost accumulation alone left them unchanged.
FP32_TRACE_MIN = 1.0      # problems that take the fp64 decisions (64-problem C5 case)
FP32_TRACE_MIN_SAMPLE = 63 / 64  # the batch-4103 sample of test_gpu_variants.py: one fp32
                                 # decision may flip near its threshold (not two)
FP32_J_TOL = 5e-3         # relative cost error of those problems, worst case
FP32_J_MEDIAN_TOL = 5e-5  # ... and typical
# Trajectories, gains and value gradients of the same-trace problems against the fp64 oracle,
# as norms relative to the oracle's per problem and phase-concatenated array:
# e = ||a - b||_inf / max(1, ||b||_inf).  Stated target (round 5) for every array: the median
# problem within 5e-3 and 95 % of the problems within 1e-2 (= the bulk of a batch accurate to
# 1 %); a single ill-conditioned problem may reach 1e-1.  Why a distribution target: the error
# of a problem is its conditioning times fp32's rounding -- the fp64 oracle's own answer moves
# by up to 7.8e-5 (X) / 2.8e-4 (G) when only x0 is rounded to float (6e-8 relative), i.e. the
# solve amplifies an input perturbation ~10^3-5x10^3 on its worst problems, and fp32
# arithmetic perturbs every knot, not just x0 (tools/diag_fp32_x0.py: x0 rounding is not a
# visible part of the fp32 error).  Measured (round 5, 64 problems): X median 2.2e-3 p95
# 7.9e-3 max 1.9e-2; U 3.7e-4 / 2.2e-3 / 8.2e-3; K 3.4e-3 / 8.6e-3 / 1.1e-2; DU 4.8e-4 /
# 1.1e-3 / 6.8e-3; G 1.3e-3 / 3.6e-3 / 6.2e-2 (one problem).
FP32_ARRAY_MEDIAN = 5e-3
FP32_ARRAY_P95 = 1e-2
FP32_ARRAY_MAX = 1e-1
FP32_ARRAYS = ("X", "U", "K", "DU", "G")


def test_c5_fp32_vs_fp64_oracle(need_gpu):
    import oracle as O
    if not O.available():
        pytest.skip("oracle not built")
    from mhpc_minimal_env_amd import configs, locomotion as L
    B = 64
    desc32 = configs.c5f32_desc()
    x0 = configs.x0_for(desc32, B)
    loco = L.MHPCLocomotion(desc=desc32, option=L.HSDDP_OPTION(), batch=B, device=0)
    loco.set_initial_condition(x0)
    loco.initialization()
    status = loco.solve_mhpc().copy()
    sc = loco.get_scalars()
    got = loco.concatenated()
    loco.close()
    ref = O.solve(configs.c5_desc(64), L.HSDDP_OPTION().to_c(), x0, nthreads=8)
    assert np.isfinite(sc["J"]).all()
    same = (sc["trace"] == ref["trace"]).all(axis=1)
    rel = np.abs(sc["J"] - ref["J"]) / np.maximum(1.0, np.abs(ref["J"]))
    print(f"fp32 C5: trace identical for {same.mean():.3f} of {B}, J rel err median "
          f"{np.median(rel):.2e}, same-trace max {rel[same].max() if same.any() else 0:.2e}, "
          f"status {np.bincount(status)}")
    assert same.mean() >= FP32_TRACE_MIN
    assert rel[same].max() <= FP32_J_TOL
    assert np.median(rel[same]) <= FP32_J_MEDIAN_TOL
    # trajectories, gains and value gradients (verdict r3: not only J)
    for k in FP32_ARRAYS:
        a = np.asarray(got[k], float)[same]
        b = np.asarray(ref[k], float)[same]
        err = np.abs(a - b).max(axis=1) / np.maximum(1.0, np.abs(b).max(axis=1))
        med, p95 = np.median(err), np.quantile(err, 0.95)
        print(f"fp32 C5 {k}: rel err median {med:.2e} p95 {p95:.2e} max {err.max():.2e}")
        assert med <= FP32_ARRAY_MEDIAN, (k, med)
        assert p95 <= FP32_ARRAY_P95, (k, p95)
        assert err.max() <= FP32_ARRAY_MAX, (k, err.max())
