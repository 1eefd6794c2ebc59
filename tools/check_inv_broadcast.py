"""Build-time check of the backward sweep's inverse broadcast (mhpc_bws.hip, R45 of
riccati_knot; round-2 review "weak 5").

Lanes 0..15 of a wave store one entry each of the 4x4 control-block inverse to LDS
(`sh.inv[lane]`, spare lanes to a junk slot) and every lane then reads all 16 entries back,
with no barrier in a one-wave block: correct because a wave's LDS operations complete in
issue order AND the compiler keeps the 16 loads behind the store (they may alias it in
per-lane semantics).  An explicit wave barrier or fence costs ~9 % of the sweep
(profiles/r02_ab_inverse_broadcast.txt), so instead this check pins the second condition in
the shipping device assembly:

  in a k_bws kernel, every `v_div_fixup_f64` result (optionally widened by
  `v_cvt_f64_f32`) stored by `ds_write_b64` is an inverse-broadcast site (the sweep stores
  no other quotient to LDS), and must be followed within the same straight-line block by
  reads covering one contiguous 128-byte window (16 doubles), none of which is issued
  before the store.  Reported: a store whose window is incomplete after it, a read of the
  window ahead of the store, and a k_bws kernel with no site at all.

usage: python tools/check_inv_broadcast.py file.s [...]   (exit 1 on a finding)"""
import re
import sys

FUNC = re.compile(r"^(_Z\w*k_bws\w*):")
ANYFUNC = re.compile(r"^([_A-Za-z][\w.$]*):")
LABEL = re.compile(r"^\.LBB\d+_\d+:")
DIV = re.compile(r"^v_div_fixup_f(64|32)\s+(v\[(\d+):(\d+)\]|v(\d+)),")
CVT = re.compile(r"^v_cvt_f64_f32(_e32|_e64)?\s+v\[(\d+):\d+\],\s*v(\d+)")
WRITE = re.compile(r"^ds_write_b64\s+v\d+,\s*v\[(\d+):\d+\]")
READ = re.compile(r"^ds_read_b(64|128)\s+v\[\d+:\d+\],\s*(v\d+)(?:\s+offset:(\d+))?")
READ2 = re.compile(r"^ds_read2_b64\s+v\[\d+:\d+\],\s*(v\d+)\s+offset0:(\d+)\s+offset1:(\d+)")
END = ("s_cbranch", "s_branch", "s_endpgm", "s_setpc")
WINDOW = 128
SCAN = 120  # instructions scanned on either side of a store


def code(line):
    return line.split(";")[0].strip()


def reads(s):
    """[(base vgpr, byte offset, size)] of one LDS read instruction (empty if none)."""
    m = READ.match(s)
    if m:
        return [(m.group(2), int(m.group(3) or 0), int(m.group(1)) // 8)]
    m = READ2.match(s)
    if m:
        return [(m.group(1), int(m.group(2)) * 8, 8), (m.group(1), int(m.group(3)) * 8, 8)]
    return []


def window(rs):
    """(base, start) of a fully covered 128-byte window among reads rs, or None."""
    by = {}
    for base, off, size in rs:
        by.setdefault(base, set()).update(range(off, off + size))
    for base, cov in by.items():
        for start in sorted(o for o in cov if o % 16 == 0):
            if all(b in cov for b in range(start, start + WINDOW)):
                return base, start
    return None


def block(lines, i, step):
    """Code lines of the straight-line block from line i (exclusive) in direction step."""
    out, k = [], i + step
    while 0 <= k < len(lines) and len(out) < SCAN:
        s = code(lines[k])
        if LABEL.match(lines[k]) or ANYFUNC.match(lines[k]):
            break
        if s:
            if s.startswith(END):
                break
            out.append(s)
        k += step
    return out


def scan(path):
    lines = open(path).read().splitlines()
    sites, bad = {}, []
    func = None
    for i, ln in enumerate(lines):
        fm = ANYFUNC.match(ln)
        if fm and not ln.startswith("."):
            func = fm.group(1) if FUNC.match(ln) else None
        if func is None:
            continue
        m = WRITE.match(code(ln))
        if not m:
            continue
        # the stored value: a division result, directly or widened from fp32
        src = int(m.group(1))
        prev = block(lines, i, -1)
        div = False
        for s in prev[:24]:
            c = CVT.match(s)
            if c and int(c.group(2)) == src:
                src = int(c.group(3))
                continue
            d = DIV.match(s)
            if d:
                lo = int(d.group(3) if d.group(3) is not None else d.group(5))
                if lo == src:
                    div = True
                    break
        if not div:
            continue
        after = [r for s in block(lines, i, 1) for r in reads(s)]
        w = window(after)
        if w is None:
            # the sweep stores no other division result to LDS: a store whose read-back is
            # incomplete after it had (some of) its reads moved above it
            bad.append((func, i + 1, "division result stored to LDS without all 16 reads "
                                     "of a 128-byte window after it in the same block"))
            continue
        base, start = w
        early = [r for s in prev for r in reads(s)
                 if r[0] == base and start <= r[1] < start + WINDOW]
        if early:
            bad.append((func, i + 1, f"{len(early)} read(s) of the window at offset {start} "
                                     f"issued before the store"))
        sites[func] = sites.get(func, 0) + 1
    return sites, bad


def main(paths):
    nbad, total = 0, 0
    for p in paths:
        sites, bad = scan(p)
        for func, line, msg in bad:
            nbad += 1
            print(f"{p}:{line}: {func}: {msg}")
        lines = open(p).read().splitlines()
        funcs = [FUNC.match(ln).group(1) for ln in lines if FUNC.match(ln)]
        for f in funcs:
            n = sites.get(f, 0)
            total += n
            if n == 0:
                nbad += 1
                print(f"{p}: {f}: no complete inverse-broadcast site (store, then 16 reads)")
    print(f"{total} inverse-broadcast site(s) in order, {nbad} finding(s)")
    return 1 if nbad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
