"""Per-part cycle breakdown of the line-search rollout's WB knots (needs a -DMHPC_RO_TIMING
build): python tools/ro_timing.py <lib.so> [batch]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["MHPC_AMD_LIB"] = sys.argv[1]
from mhpc_minimal_env_amd import capi, configs, locomotion as L  # noqa: E402

B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
lib = capi.lib()
dbg = lib.mhpc_dbg_ro_cycles
dbg.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
desc = configs.c3_desc()
loco = L.MHPCLocomotion(desc=desc, option=L.HSDDP_OPTION(), batch=B, device=0)
loco.set_initial_condition(configs.x0_for(desc, B))
buf = (ctypes.c_ulonglong * 5)()
for it in range(2):
    loco.initialization()
    dbg(buf, 1)
    loco.solve_mhpc()
    dbg(buf, 1)
c = list(buf)
n = c[4]
print("batch", B, "WB knots timed (wave lane 0):", n)
for name, v in zip(["feedback u", "wb_dynamics", "running cost", "store + step"], c[:4]):
    print(f"{name:14s} {v / n:9.1f} cyc/knot")
print(f"{'total':14s} {sum(c[:4]) / n:9.1f} cyc/knot")
