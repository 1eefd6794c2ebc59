"""fp32 C5 against the fp64 oracle: with the exact x0 and with x0 rounded to float (the input
the fp32 instantiation actually solves from), and the fp64 oracle's own sensitivity to that
rounding -- how much of the fp32 array error is the problem's conditioning."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
from mhpc_minimal_env_amd import configs, locomotion as L  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
desc32 = configs.c5f32_desc()
d64 = configs.c5_desc(64)
x0 = configs.x0_for(desc32, B)
x0f = x0.astype(np.float32).astype(np.float64)
loco = L.MHPCLocomotion(desc=desc32, option=L.HSDDP_OPTION(), batch=B, device=0)
loco.set_initial_condition(x0)
loco.initialization()
loco.solve_mhpc()
got = loco.concatenated()
got.update(loco.get_scalars())
loco.close()
opt = L.HSDDP_OPTION().to_c()
ref = O.solve(d64, opt, x0, nthreads=16)
reff = O.solve(d64, opt, x0f, nthreads=16)


def err(a, b, same):
    a = np.asarray(a, float)[same]
    b = np.asarray(b, float)[same]
    return np.abs(a - b).max(axis=1) / np.maximum(1.0, np.abs(b).max(axis=1))


for name, r in (("oracle x0", ref), ("oracle float(x0)", reff)):
    same = (got["trace"] == r["trace"]).all(axis=1)
    print(f"fp32 vs {name}: traces {same.sum()}/{B}")
    for k in ("X", "U", "K", "DU", "G"):
        e = err(got[k], r[k], same)
        print(f"  {k}: median {np.median(e):.2e} p95 {np.quantile(e, .95):.2e} max {e.max():.2e} (problem {np.argmax(e)})")
same = (ref["trace"] == reff["trace"]).all(axis=1)
print(f"fp64 oracle x0 vs float(x0): traces {same.sum()}/{B}")
for k in ("X", "U", "K", "DU", "G"):
    e = err(reff[k], ref[k], same)
    print(f"  {k}: median {np.median(e):.2e} p95 {np.quantile(e, .95):.2e} max {e.max():.2e} (problem {np.argmax(e)})")
