"""C5 fp64 (64 problems): per-phase cost of the fused unstaged line search vs the pair variant
under different run-time options (no codegen change).  MHPC_AMD_LIB selects the build."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT]
from mhpc_minimal_env_amd import configs, locomotion as L  # noqa: E402

desc = configs.c5_desc(64)
B = 64
x0 = configs.x0_for(desc, B, offset=7000)
OPTS = {"default": {}, "AL_off": {"AL_active": 0}, "AL1": {"max_AL_iter": 1},
        "ReB_off": {"ReB_active": 0}, "AL1_DDP1": {"max_AL_iter": 1, "max_DDP_iter": 1}}
out = {}
for name, kw in OPTS.items():
    res = {}
    for ro in ("pair", "fused"):
        opt = L.HSDDP_OPTION()
        for k, v in kw.items():
            setattr(opt, k, v)
        lo = L.MHPCLocomotion(desc=desc, option=opt, batch=B, device=0)
        lo.set_kernel_variant(rollout=ro)
        lo.set_initial_condition(x0)
        lo.initialization()
        lo.solve_mhpc()
        o = lo.concatenated()
        o.update(lo.get_scalars())
        lo.close()
        res[ro] = o
    a, b = res["pair"], res["fused"]
    dV = np.asarray(b["V"]) - np.asarray(a["V"])
    same = [k for k in ("X", "U", "K", "viol", "trace") if np.array_equal(np.asarray(a[k]), np.asarray(b[k]))]
    print(f"{name}: bitwise {same}; phases with a V diff {np.nonzero(np.abs(dV).max(0))[0].tolist()}; "
          f"problems {int((dV != 0).any(1).sum())}; dV3[:8] {np.round(dV[:8, 3], 6).tolist()}")
    for k in ("V", "J", "viol"):
        out[f"{name}_{k}_pair"] = np.asarray(a[k]); out[f"{name}_{k}_fused"] = np.asarray(b[k])
    off = (80 + 100 + 80) * 14 + 99 * 14
    out[f"{name}_xe3"] = np.asarray(a["X"])[:, off:off + 14]
    out[f"{name}_trace"] = np.asarray(a["trace"])
np.savez(sys.argv[1], **out)
