"""The build gate against the gfx950 register-allocator miscompile found in round 3
(DESIGN.md §5): a live-range copy placed ahead of the EXEC restore of a divergent join block
runs for no lane when the branch before it was skipped.  The checker must flag that shape,
pass the legal placements, and pass every kernel TU of the shipping build.  The same gate pins
the order of the sweep's barrier-free inverse broadcast (round-2 review, weak 5): the 16 LDS
reads of the inverse must follow the lane-0..15 store in every k_bws kernel."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import check_exec_prologue as C  # noqa: E402
import check_inv_broadcast as I  # noqa: E402

CSRC = os.path.join(ROOT, "mhpc_minimal_env_amd", "csrc")


def test_checker_flags_the_miscompile_shape_only():
    hits = C.scan(os.path.join(ROOT, "tests", "golden", "isa_join_copy.s"))
    assert [(h[0], h[1], h[3]) for h in hits] == [("bad_kernel", ".LBB0_4", [168, 169])]


def test_inverse_broadcast_checker_flags_hoisted_reads():
    """tests/golden/isa_inv_broadcast.s: one site as the shipping build emits it and two copies
    with one / all of the window's reads moved above the store."""
    sites, bad = I.scan(os.path.join(ROOT, "tests", "golden", "isa_inv_broadcast.s"))
    assert sites == {"_ZN4mhpc5k_bwsILi64ELi2ELi1EEEvgood": 1}
    assert sorted(b[0].rsplit("Ev", 1)[1] for b in bad) == ["all_reads_hoisted", "one_read_hoisted"]


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")
def test_shipping_kernels_have_no_misplaced_join_copy():
    r = subprocess.run(["make", "-j4", "-C", CSRC, "isa-check"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    isa = [os.path.join(CSRC, "_build", f) for f in ("kernels.s", "bws.s", "kernels32.s", "bws32.s")]
    assert C.scan_all(isa) == []
    sweeps = [os.path.join(CSRC, "_build", f) for f in ("bws.s", "bws32.s")]
    assert I.main(sweeps) == 0
    for p in sweeps:  # two knot kinds (or one) in each of the seven k_bws instantiations
        sites, _ = I.scan(p)
        assert len(sites) == 7 and all(n >= 1 for n in sites.values()), sites
