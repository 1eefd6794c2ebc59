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
FP32_TRACE_MIN_SAMPLE = 62 / 64  # the batch-4103 sample of test_gpu_variants.py (ADVICE r3:
                                 # one harmless codegen change may flip a single fp32 decision)
FP32_J_TOL = 5e-3         # relative cost error of those problems, worst case
FP32_J_MEDIAN_TOL = 5e-5  # ... and typical
# Trajectories, gains and value gradients of the same-trace problems against the fp64 oracle,
# as norms relative to the oracle's per problem and phase-concatenated array:
# ||a - b||_inf / max(1, ||b||_inf); worst case over the problems.  Measured (round 4, 64
# problems): X median 2.4e-3 max 2.1e-2, U 4.2e-4 / 3.5e-3, K 2.8e-3 / 9.5e-3, DU 4.1e-4 /
# 2.4e-3, G (value gradient) 1.1e-3 / 2.2e-2; bounds ~2.5x the worst case
FP32_ARRAY_TOL = {"X": 5e-2, "U": 1e-2, "K": 2.5e-2, "DU": 1e-2, "G": 5e-2}


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
    for k, tol in FP32_ARRAY_TOL.items():
        a = np.asarray(got[k], float)[same]
        b = np.asarray(ref[k], float)[same]
        err = np.abs(a - b).max(axis=1) / np.maximum(1.0, np.abs(b).max(axis=1))
        print(f"fp32 C5 {k}: rel err median {np.median(err):.2e} max {err.max():.2e}")
        assert err.max() <= tol, (k, err.max())
