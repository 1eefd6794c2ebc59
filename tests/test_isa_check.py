"""The build gate against the gfx950 register-allocator miscompile found in round 3
(DESIGN.md §5): a live-range copy placed ahead of the EXEC restore of a divergent join block
runs for no lane when the branch before it was skipped.  The checker must flag that shape,
pass the legal placements, and pass every kernel TU of the shipping build."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import check_exec_prologue as C  # noqa: E402

CSRC = os.path.join(ROOT, "mhpc_minimal_env_amd", "csrc")


def test_checker_flags_the_miscompile_shape_only():
    hits = C.scan(os.path.join(ROOT, "tests", "golden", "isa_join_copy.s"))
    assert [(h[0], h[1], h[3]) for h in hits] == [("bad_kernel", ".LBB0_4", [168, 169])]


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")
def test_shipping_kernels_have_no_misplaced_join_copy():
    r = subprocess.run(["make", "-j4", "-C", CSRC, "isa-check"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    isa = [os.path.join(CSRC, "_build", f) for f in ("kernels.s", "bws.s", "kernels32.s", "bws32.s")]
    assert C.scan_all(isa) == []
