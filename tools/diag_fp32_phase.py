"""fp32 C5 vs the fp64 oracle per phase: is the cost error an evaluation error (same
trajectory, different cost) or a different iterate (trajectory / gains differ)?"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
from mhpc_minimal_env_amd import configs, locomotion as L  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
desc = configs.c5_desc(32)
x0 = configs.x0_for(desc, B)
loco = L.MHPCLocomotion(desc=desc, option=L.HSDDP_OPTION(), batch=B, device=0)
loco.set_initial_condition(x0)
loco.initialization()
loco.solve_mhpc()
sc = loco.get_scalars()
parts = [loco.get_phase(p) for p in range(desc.n_phases)]
loco.close()
d64 = configs.c5_desc(64)
ref = O.solve(d64, L.HSDDP_OPTION().to_c(), x0, nthreads=8)
rel = np.abs(sc["J"] - ref["J"]) / np.abs(ref["J"])
off = {"X": 0, "U": 0, "K": 0}
refp = []
for p in range(desc.n_phases):
    n, N = desc.xsize(p), desc.N[p]
    q = {}
    for k, w in (("X", n), ("U", 4), ("K", 4 * n)):
        q[k] = ref[k][:, off[k]:off[k] + N * w].reshape(B, N, w)
        off[k] += N * w
    refp.append(q)
for i in np.argsort(-rel)[:3]:
    print(f"problem {i}: J rel err {rel[i]:.2e}")
    for p in range(desc.n_phases):
        g = parts[p]
        dx = np.max(np.abs(g["x"][i] - refp[p]["X"][i]))
        du = np.max(np.abs(g["u"][i] - refp[p]["U"][i]))
        dk = np.max(np.abs(g["K"][i].reshape(desc.N[p], -1) - refp[p]["K"][i])) / max(1e-30, np.max(np.abs(refp[p]["K"][i])))
        dV = (sc["V"][i, p] - ref["V"][i, p]) / abs(ref["V"][i, p])
        print(f"  phase {p}: max|dx| {dx:.2e} max|du| {du:.2e} K rel {dk:.2e}  V rel {dV:+.2e}")
