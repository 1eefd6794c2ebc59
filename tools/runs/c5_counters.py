import sys; sys.path.insert(0, '.')
from mhpc_minimal_env_amd import configs, locomotion as L
for prec in (64, 32):
    desc = configs.c5_desc(prec)
    B = 4096
    loco = L.MHPCLocomotion(desc=desc, option=L.HSDDP_OPTION(), batch=B, device=0)
    loco.set_initial_condition(configs.x0_for(desc, B)); loco.initialization(); loco.solve_mhpc()
    print(prec, loco.get_counters()); loco.close()
