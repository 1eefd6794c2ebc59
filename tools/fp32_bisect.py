"""fp32 accuracy of C5 across builds (bisect the round-5 fp32 regression).

  python tools/fp32_bisect.py <out.json> <tree> [<tree> ...]

Each <tree> is a source tree holding its own `mhpc_minimal_env_amd` package with a built
libmhpc_amd.so (an older commit's, extracted and built by hand).  Every tree solves the same
64-problem C5 fp32 batch (configs.x0_for) in a process of its own with that tree's package;
this process then compares each result with the fp64 oracle of the current tree (the checker:
test infrastructure only) the way tests/test_gpu_fp32.py does -- per problem
||a - b||_inf / max(1, ||b||_inf) of the phase-concatenated arrays -- and prints median, 95th
percentile, max and the worst problem per array."""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = ("X", "U", "K", "DU", "G", "J", "trace", "status")
B = 64

_CHILD = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from mhpc_minimal_env_amd import configs, locomotion as L
d = configs.c5_desc(32)
x0 = configs.x0_for(d, %d)
lo = L.MHPCLocomotion(desc=d, option=L.HSDDP_OPTION(), batch=%d, device=0)
lo.set_initial_condition(x0)
lo.initialization()
st = lo.solve_mhpc().copy()
o = lo.concatenated()
o.update(lo.get_scalars())
o["status"] = st
lo.close()
np.savez(sys.argv[2], **{k: np.asarray(o[k]) for k in %r})
""" % (B, B, KEYS)


def oracle_ref():
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from mhpc_minimal_env_amd import configs, locomotion as L
    d = configs.c5_desc(64)
    x0 = configs.x0_for(d, B)
    return O.solve(d, L.HSDDP_OPTION().to_c(), x0, nthreads=8)


def stats(got, ref):
    same = (got["trace"] == ref["trace"]).all(axis=1)
    rel = np.abs(got["J"] - ref["J"]) / np.maximum(1.0, np.abs(ref["J"]))
    out = {"trace_same": int(same.sum()), "J_med": float(np.median(rel[same])),
           "J_max": float(rel[same].max())}
    for k in ("X", "U", "K", "DU", "G"):
        a = np.asarray(got[k], float)[same]
        b = np.asarray(ref[k], float)[same]
        err = np.abs(a - b).max(axis=1) / np.maximum(1.0, np.abs(b).max(axis=1))
        idx = np.where(same)[0]
        out[k] = {"med": float(np.median(err)), "p95": float(np.quantile(err, 0.95)),
                  "max": float(err.max()), "worst": int(idx[int(err.argmax())]),
                  "top3": [int(idx[i]) for i in np.argsort(err)[::-1][:3]]}
    return out


def main(out_json, trees):
    ref = oracle_ref()
    res = {}
    for t in trees:
        with tempfile.TemporaryDirectory() as td:
            f = os.path.join(td, "o.npz")
            env = dict(os.environ)
            env.pop("MHPC_AMD_LIB", None)
            r = subprocess.run([sys.executable, "-c", _CHILD, os.path.abspath(t), f], env=env,
                               capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                print(t, "FAILED", r.stderr[-2000:], flush=True)
                res[t] = {"error": r.stderr[-2000:]}
                continue
            got = dict(np.load(f))
        s = stats(got, ref)
        res[t] = s
        print(f"{os.path.basename(t.rstrip('/')):>10}: traces {s['trace_same']}/{B} J med {s['J_med']:.1e} "
              f"max {s['J_max']:.1e} | " + " ".join(
                  f"{k} {s[k]['med']:.1e}/{s[k]['p95']:.1e}/{s[k]['max']:.1e}@{s[k]['worst']}"
                  for k in ("X", "U", "K", "DU", "G")), flush=True)
    with open(out_json, "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
