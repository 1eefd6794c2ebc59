import sys, numpy as np
sys.path[:0] = ['.', 'oracle', 'tests']
from mhpc_minimal_env_amd import configs, locomotion as L
import oracle as O
from test_gpu_solve import run_gpu
desc, opt = configs.c3_desc(), L.HSDDP_OPTION()
for B in (7, 8, 1, 3):
    x0 = configs.x0_for(desc, B)
    got = run_gpu(desc, opt, x0)
    ref = O.solve(desc, opt.to_c(), x0, nthreads=8)
    for b in range(B):
        e = np.max(np.abs(got["X"][b] - ref["X"][b]))
        tr = (got["trace"][b] == ref["trace"][b]).all()
        if e > 1e-6 or not tr:
            print("B", B, "prob", b, "Xerr", e, "trace ok", tr, "nz first", got["X"][b][:3], O.decode_trace(got["trace"][b]))
    print("B", B, "done")
