"""C5 fp64, 64 problems: the fused unstaged line search (k_rollout<false,false,false>) vs the
pair variant and the oracle, per phase cost.  MHPC_AMD_LIB selects the build.
python tools/repro_cw/diag_cw.py out.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
from mhpc_minimal_env_amd import configs, locomotion as L  # noqa: E402

desc = configs.c5_desc(64)
B = 64
x0 = configs.x0_for(desc, B, offset=7000)
res = {}
for ro in ("pair", "fused"):
    lo = L.MHPCLocomotion(desc=desc, option=L.HSDDP_OPTION(), batch=B, device=0)
    lo.set_kernel_variant(rollout=ro)
    lo.set_initial_condition(x0)
    lo.initialization()
    lo.solve_mhpc()
    o = lo.concatenated()
    o.update(lo.get_scalars())
    lo.close()
    res[ro] = o
a, b = res["pair"], res["fused"]
for k in ("X", "U", "Y", "K", "DU", "G", "J", "V", "dV", "viol", "trace"):
    same = np.array_equal(np.asarray(a[k]), np.asarray(b[k]))
    print(k, "bitwise" if same else "DIFFERS")
dV = np.asarray(b["V"]) - np.asarray(a["V"])
print("V diff per phase (max abs):", np.abs(dV).max(0))
print("problems with a V diff:", int((dV != 0).any(1).sum()))
print("J diff:", (np.asarray(b["J"]) - np.asarray(a["J"]))[:8])
import oracle as O  # noqa: E402
if O.available():
    ref = O.solve(desc, L.HSDDP_OPTION().to_c(), x0, nthreads=8)
    for ro in ("pair", "fused"):
        e = np.abs(np.asarray(res[ro]["J"]) - ref["J"]) / np.maximum(1, np.abs(ref["J"]))
        print(ro, "J rel err vs oracle", float(e.max()))
np.savez(sys.argv[1] if len(sys.argv) > 1 else "diag_cw.npz",
         **{f"{ro}_{k}": np.asarray(res[ro][k]) for ro in res for k in ("J", "V", "viol", "trace")})
