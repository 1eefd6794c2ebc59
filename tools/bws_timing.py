"""Per-part cycle breakdown of the backward sweep (needs a -DMHPC_BWS_TIMING build):
python tools/bws_timing.py <lib.so> [batch] [variant]   (clock64 on lane 0 of every wave)"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["MHPC_AMD_LIB"] = sys.argv[1]
from mhpc_minimal_env_amd import capi, configs, locomotion as L  # noqa: E402

B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
var = sys.argv[3] if len(sys.argv) > 3 else "auto"
lib = capi.lib()
dbg = lib.mhpc_dbg_bws_cycles
dbg.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
desc = configs.c3_desc()
loco = L.MHPCLocomotion(desc=desc, option=L.HSDDP_OPTION(), batch=B, device=0)
loco.set_kernel_variant(bws=var)
loco.set_initial_condition(configs.x0_for(desc, B))
buf = (ctypes.c_ulonglong * 16)()
for it in range(2):
    loco.initialization()
    dbg(buf, 1)
    loco.solve_mhpc()
    dbg(buf, 1)
c = list(buf)
waves = max(c[7], 1)
print(f"batch {B} bws={var}: {c[7]} wave launches, per wave:")
print(f"  kernel        {c[6] / waves:10.0f} cyc")
print(f"  WB knots      {c[0] / waves:10.0f} cyc  {c[1] / waves:6.1f} knots  {c[0] / max(c[1], 1):7.0f} cyc/knot")
print(f"  SRB knots     {c[2] / waves:10.0f} cyc  {c[3] / waves:6.1f} knots  {c[2] / max(c[3], 1):7.0f} cyc/knot")
print(f"  terminal      {c[4] / waves:10.0f} cyc")
print(f"  impact        {c[5] / waves:10.0f} cyc")
nk = max(c[3], 1)
segs = ("operands / stores", "S and Q", "Qxx transpose (LDS)", "control block", "value update")
print("  SRB knot segments (instrumented, per knot):")
for i, name in enumerate(segs):
    print(f"    {name:22s} {c[8 + i] / nk:7.0f} cyc")
