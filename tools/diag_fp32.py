"""fp32 C5 vs the fp64 oracle: trace divergence rate and cost error."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
from mhpc_minimal_env_amd import configs, locomotion as L  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
for prec in (64, 32):
    desc = configs.c5_desc(prec)
    x0 = configs.x0_for(desc, B)
    loco = L.MHPCLocomotion(desc=desc, option=L.HSDDP_OPTION(), batch=B, device=0)
    loco.set_initial_condition(x0)
    loco.initialization()
    st = loco.solve_mhpc().copy()
    sc = loco.get_scalars()
    loco.close()
    ref = O.solve(configs.c5_desc(64), L.HSDDP_OPTION().to_c(), x0, nthreads=8)
    same = (sc["trace"] == ref["trace"]).all(axis=1)
    rel = np.abs(sc["J"] - ref["J"]) / np.abs(ref["J"])
    print(f"precision {prec}: status {np.bincount(st)}, trace identical {same.mean():.3f}, "
          f"J rel err median {np.median(rel):.2e} max {rel.max():.2e} "
          f"(same-trace max {rel[same].max() if same.any() else float('nan'):.2e}), finite {np.isfinite(sc['J']).all()}")
    if prec == 32:
        w = np.argsort(-rel)[:4]
        for i in w:
            print(f"  problem {i}: J fp32 {sc['J'][i]:.6g} oracle {ref['J'][i]:.6g} viol {sc['viol'][i]:.3g}/{ref['viol'][i]:.3g}")
            print("    V fp32  ", np.array2string(sc["V"][i], precision=4))
            print("    V oracle", np.array2string(ref["V"][i], precision=4))
