"""Where does fp32 C5 depart from the fp64 oracle?  Per phase, max |dx| of the nominal
trajectory (and the gains' relative error) after: the warm start only, one AL x one DDP
iteration, and the full solve (2 x 3).  Median over the batch and the worst problem."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
from mhpc_minimal_env_amd import configs, locomotion as L  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
WATCH = int(sys.argv[2]) if len(sys.argv) > 2 else -1  # one problem to report per phase
desc = configs.c5_desc(32)
d64 = configs.c5_desc(64)
x0 = configs.x0_for(desc, B)
P = desc.n_phases


def split(a, w_of):
    out, o = [], 0
    for p in range(P):
        w = w_of(p) * desc.N[p]
        out.append(a[:, o:o + w])
        o += w
    return out


for name, al, ddp, solve in (("warm start", 2, 3, False), ("AL1 x DDP1", 1, 1, True),
                             ("AL1 x DDP3", 1, 3, True), ("full 2 x 3", 2, 3, True)):
    opt = L.HSDDP_OPTION()
    opt.max_AL_iter, opt.max_DDP_iter = al, ddp
    loco = L.MHPCLocomotion(desc=desc, option=opt, batch=B, device=0)
    loco.set_initial_condition(x0)
    loco.initialization()
    if solve:
        loco.solve_mhpc()
    g = loco.concatenated()
    sc = loco.get_scalars()
    loco.close()
    ref = O.solve(d64, opt.to_c(), x0, nthreads=8, do_solve=solve)
    gx, rx = split(g["X"], desc.xsize), split(ref["X"], desc.xsize)
    gk, rk = split(g["K"], lambda p: 4 * desc.xsize(p)), split(ref["K"], lambda p: 4 * desc.xsize(p))
    gg, rg = split(g["G"], desc.xsize), split(ref["G"], desc.xsize)
    same = (sc["trace"] == ref["trace"]).all(axis=1).mean() if solve else 1.0
    rel = np.abs(sc["J"] - ref["J"]) / np.abs(ref["J"]) if solve else np.zeros(B)
    print(f"== {name}: traces {same:.3f}, J rel err median {np.median(rel):.1e} max {rel.max():.1e}")
    for p in range(P):
        dx = np.max(np.abs(gx[p] - rx[p]), axis=1)
        kr = np.max(np.abs(gk[p] - rk[p]), axis=1) / np.maximum(1e-30, np.max(np.abs(rk[p]), axis=1))
        gr = np.max(np.abs(gg[p] - rg[p]), axis=1) / np.maximum(1.0, np.max(np.abs(rg[p]), axis=1))
        w = (f"   problem {WATCH}: dx {dx[WATCH]:.1e} K {kr[WATCH]:.1e} G {gr[WATCH]:.1e} "
             f"(|G|max {np.abs(rg[p][WATCH]).max():.1e})") if WATCH >= 0 else ""
        print(f"   phase {p}: max|dx| median {np.median(dx):.1e} worst {dx.max():.1e}   "
              f"K rel median {np.median(kr):.1e} worst {kr.max():.1e}   G worst {gr.max():.1e}" + w)
