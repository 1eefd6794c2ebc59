"""Per-round cycle breakdown of k_bws (needs a -DMHPC_BWS_TIMING build, see
tools/build_variants.sh): python tools/bws_timing.py <lib.so> [batch]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["MHPC_AMD_LIB"] = sys.argv[1]
from mhpc_minimal_env_amd import capi, configs, locomotion as L  # noqa: E402

B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
lib = capi.lib()
dbg = lib.mhpc_dbg_bws_cycles
dbg.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
desc = configs.c3_desc()
loco = L.MHPCLocomotion(desc=desc, option=L.HSDDP_OPTION(), batch=B, device=0)
# the round marks sit in the whole-sweep kernel (PART 0): no split at the WB / SRB boundary
loco.set_kernel_variant(overlap="off")
loco.set_initial_condition(configs.x0_for(desc, B))
buf = (ctypes.c_ulonglong * 12)()
for it in range(2):
    loco.initialization()
    dbg(buf, 1)
    loco.solve_mhpc()
    dbg(buf, 1)
c = loco.get_counters()
cyc = np.array(list(buf), dtype=np.float64)
names = ["total", "WB R2 side (stores/load)", "WB R3", "WB R2 compute", "SRB R2 compute",
         "WB R45 compute", "SRB R45 compute", "WB R45 side (drop)",
         "SRB R2 side (stores/load)", "SRB R3", "SRB R45 side (drop)", ""]
knots = c["bws_knots"]
print("batch", B, "counters", c)
print(f"{'round':24s} {'cyc/problem':>12s} {'cyc/knot':>10s} {'share':>7s}")
# C3: half of the swept knots are WB, half SRB (per-kind cycles / (knots / 2))
for i in [0, 3, 1, 2, 5, 7, 4, 8, 9, 6, 10]:
    kn = knots if i == 0 else knots / 2
    print(f"{names[i]:24s} {cyc[i]/B:12.0f} {cyc[i]/kn:10.1f} {cyc[i]/cyc[0]:7.3f}")
rest = cyc[0] - cyc[1:11].sum()
print(f"{'other (terminal/impact)':24s} {rest/B:12.0f} {rest/knots:10.1f} {rest/cyc[0]:7.3f}")
