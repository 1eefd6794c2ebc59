"""The build gates on device assembly (csrc/Makefile, _build/isa.ok):
  * the gfx950 register-allocator miscompile found in round 3: a live-range copy
    placed ahead of the EXEC restore of a divergent join block runs for no lane when the branch
    before it was skipped -- the checker must flag that shape and pass the legal placements;
  * DPP read-after-write hazards (round 4): the sweep's row-broadcast multiply-adds are inline
    assembly (mhpc_dpp.h), outside the compiler's hazard recognizer; a DPP instruction may not
    read a VGPR written in the previous 2 wait states;
  * no scratch memory in the solve's kernels (round 4): a scratch access waits on gfx950's
    single in-order VM counter behind every earlier global store.
All must pass every kernel TU of the shipping build."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import check_exec_prologue as C  # noqa: E402
import check_dpp_hazards as D  # noqa: E402
import check_no_scratch as S  # noqa: E402

CSRC = os.path.join(ROOT, "mhpc_minimal_env_amd", "csrc")


def test_checker_flags_the_miscompile_shape_only():
    hits = C.scan(os.path.join(ROOT, "tests", "golden", "isa_join_copy.s"))
    assert [(h[0], h[1], h[3]) for h in hits] == [("bad_kernel", ".LBB0_4", [168, 169])]


def test_dpp_hazard_checker(tmp_path):
    """A DPP read of a VGPR written 1 wait state earlier (source or accumulator) is flagged;
    2 wait states (s_nop 1, or two instructions) pass; a v_fmac_*_dpp right after a label
    (unknown predecessor) is flagged unless an s_nop covers it."""
    f = "row_newbcast:1 row_mask:0xf bank_mask:0xf"
    src = "\n".join([
        "good:",
        "\ts_nop 1",
        "\tv_mul_f64 v[2:3], v[0:1], v[0:1]",
        "\ts_nop 1",
        f"\tv_fmac_f64_dpp v[4:5], v[2:3], v[6:7] {f}",
        f"\tv_fmac_f64_dpp v[8:9], v[2:3], v[6:7] {f}",
        f"\tv_fmac_f64_dpp v[10:11], v[2:3], v[6:7] {f}",
        f"\tv_fmac_f64_dpp v[4:5], v[2:3], v[6:7] {f}",
        "src_hazard:",
        "\ts_nop 1",
        "\tv_mul_f64 v[2:3], v[0:1], v[0:1]",
        "\ts_nop 0",
        f"\tv_fmac_f64_dpp v[4:5], v[2:3], v[6:7] {f}",
        "acc_hazard:",
        "\ts_nop 1",
        f"\tv_fmac_f64_dpp v[4:5], v[2:3], v[6:7] {f}",
        f"\tv_fmac_f64_dpp v[8:9], v[2:3], v[6:7] {f}",
        f"\tv_fmac_f64_dpp v[4:5], v[2:3], v[6:7] {f}",
        "label_hazard:",
        f"\tv_fmac_f64_dpp v[4:5], v[2:3], v[6:7] {f}",
        ""])
    p = tmp_path / "h.s"
    p.write_text(src)
    bad = D.check(str(p))
    assert sorted(b.split(": ")[1] for b in bad) == ["acc_hazard", "label_hazard", "src_hazard"]


def test_no_scratch_checker(tmp_path):
    """A hot kernel with a scratch instruction or a private segment is flagged; the debug-info
    kernel (not in the solve) and kernels outside the solve are not."""
    def kern(name, body, priv):
        # descriptor block as hipcc emits it, and metadata whose ".args" entries carry ".name"s
        # (which must not be taken for the kernel's name: ADVICE r4)
        return (f"{name}:\n{body}\n.Lfunc_end{name}:\n"
                f"\t.amdhsa_kernel {name}\n\t\t.amdhsa_group_segment_fixed_size 0\n"
                f"\t\t.amdhsa_private_segment_fixed_size {priv}\n\t.end_amdhsa_kernel\n",
                f"  - .args:\n      - .name: sp\n        .size: 8\n      - .name: d\n"
                f"    .name: {name}\n    .private_segment_fixed_size: {priv}\n")
    parts = [kern("_ZN4mhpc9k_rolloutILb1EEEv", "\tscratch_store_dwordx2 v0, v[2:3], off", 0),
             kern("_ZN4mhpc5k_bwsILi2EEEv", "\tv_mov_b32_e32 v0, 0", 16),
             kern("_ZN4mhpc6k_initEv", "\tv_mov_b32_e32 v0, 0", 0),
             kern("_ZN4mhpc11k_cost_gradEv", "\tscratch_load_dword v0, off, s0", 8),
             kern("_ZN4mhpc8k_exportEv", "\tscratch_load_dword v0, off, s0", 8)]
    p = tmp_path / "k.s"
    p.write_text("".join(a for a, _ in parts) + "amdhsa.kernels:\n" + "".join(b for _, b in parts))
    bad = S.check(str(p))
    assert len(bad) == 2
    assert any("k_rollout" in b and "1 scratch instructions" in b for b in bad)
    assert any("k_bws" in b and "private segment 16" in b for b in bad)


def test_generated_dpp_header_is_current():
    """mhpc_dpp.h is what tools/gen_dpp_asm.py generates."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_dpp_asm.py")],
                       capture_output=True, text=True, check=True)
    with open(os.path.join(CSRC, "mhpc_dpp.h")) as f:
        assert f.read() == r.stdout


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")
def test_shipping_kernels_have_no_misplaced_join_copy():
    r = subprocess.run(["make", "-j4", "-C", CSRC, "isa-check"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    isa = [os.path.join(CSRC, "_build", f) for f in ("kernels.s", "bws.s", "kernels32.s", "bws32.s")]
    assert C.scan_all(isa) == []
    sweeps = [os.path.join(CSRC, "_build", f) for f in ("bws.s", "bws32.s")]
    assert D.main(sweeps) == 0
    assert S.main(isa) == 0
    for p in sweeps:  # the row-broadcast FMAs are there (the gate checked something)
        with open(p) as f:
            assert f.read().count("_dpp ") > 1000
