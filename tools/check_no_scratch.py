"""Build gate: the solve's hot kernels keep everything in registers / LDS -- no private
(scratch) memory.  A scratch load or store uses the VM counter, and on gfx950's single
in-order counter a wait for it also waits for every global store issued before it (the
line search's record stores: a per-lane index into the kernel parameter block once made the
compiler copy the block to scratch and the rollout 65 % slower).  Checks the device assembly
(hipcc --cuda-device-only -S) of every kernel whose name matches HOT: no scratch_* instruction
and a zero private segment.

usage: python tools/check_no_scratch.py <file.s> [...]    exit 1 on any hit
"""
import re
import sys

HOT = ("k_rollout", "k_bws", "k_partials", "k_init", "k_cost", "k_al_end")
COLD = ("k_cost_grad",)  # debug-info kernel (print_debugInfo), not in the solve


def check(path):
    s = open(path).read()
    bad = []
    # each kernel's own descriptor block (.amdhsa_kernel <symbol> ... .end_amdhsa_kernel): the
    # metadata's ".name:" entries also name kernel arguments, so they cannot anchor the kernel
    for m in re.finditer(r"^\s*\.amdhsa_kernel\s+(\S+)\n(.*?)^\s*\.end_amdhsa_kernel", s, re.S | re.M):
        name = m.group(1)
        pm = re.search(r"\.amdhsa_private_segment_fixed_size\s+(\d+)", m.group(2))
        priv = int(pm.group(1)) if pm else 0
        if any(h in name for h in HOT) and not any(c in name for c in COLD) and priv:
            bad.append(f"{path}: {name}: private segment {priv} bytes")
    for name in re.findall(r"^(_Z\S+):", s, re.M):
        if not any(h in name for h in HOT) or any(c in name for c in COLD):
            continue
        a = s.index(name + ":")
        b = s.index(".Lfunc_end", a)
        n = len(re.findall(r"^\s*scratch_", s[a:b], re.M))
        if n:
            bad.append(f"{path}: {name}: {n} scratch instructions")
    return bad


def main(paths):
    bad = [b for p in paths for b in check(p)]
    for b in bad:
        print(b)
    print(f"check_no_scratch: {len(paths)} file(s), {len(bad)} hit(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
