"""Build-time check for the gfx950 miscompile found in round 3 ("The
codegen-sensitive line-search cost"): a register copy that the register allocator placed at
the top of a control-flow JOIN block, before the `s_or_b64 exec, exec, s[..]` that restores
the lanes of the divergent region.  Such an instruction runs with the mask of the branch that
reached the join last -- an EMPTY mask when that branch had no lanes and was skipped by
`s_cbranch_execz` -- so lanes that took the other branch never get the copy, and read a stale
register afterwards.

Instructions of the skipped branch itself may legally sit there (their results are only
used by that branch's lanes).  A placement is reported when a VGPR written there
  * is not written anywhere in the other (then-) branch of the region, and
  * is read after the exec restore before being written again (straight-line scan up to
    the next branch; a scan that reaches a branch first counts as a read, conservatively).

usage: python tools/check_exec_prologue.py file.s [...]   (exit 1 if anything is reported)
       .s from: hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S -o f.s src.hip"""
import re
import sys

LABEL = re.compile(r"^(\.LBB\d+_\d+):")
FUNC = re.compile(r"^([_A-Za-z][\w.$]*):")
RESTORE = re.compile(r"^s_or_b(64|32)\s+exec(_lo)?,\s*exec(_lo)?,")
VREG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")
NO_VDST = ("global_store", "buffer_store", "flat_store", "scratch_store", "ds_write", "ds_store",
           "v_cmp", "v_readlane", "v_readfirstlane", "v_writelane", "s_")
READS_DST = ("v_fmac", "v_mac", "v_fmamk", "v_fmaak", "v_cndmask")  # dst also read (fmac)


def regs(op):
    out = set()
    for m in VREG.finditer(op):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def decode(s):
    """(mnemonic, written VGPRs, read VGPRs) of one instruction."""
    parts = s.split(None, 1)
    mn = parts[0]
    ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
    if not ops:
        return mn, set(), set()
    if mn.startswith(NO_VDST):
        return mn, set(), set().union(*[regs(o) for o in ops])
    w = regs(ops[0])
    r = set().union(*[regs(o) for o in ops[1:]]) if len(ops) > 1 else set()
    if mn.startswith(READS_DST):
        r |= w
    return mn, w, r


COPY = ("v_mov_b32", "v_mov_b64", "v_accvgpr_read", "v_accvgpr_write", "v_accvgpr_mov")


def region_start(lines, i, target):
    """Line of the s_and_saveexec opening the divergent region that joins at line i."""
    first = i
    refs = [target]
    for k in range(i - 1, -1, -1):
        c = code(lines[k])
        if FUNC.match(lines[k]) and not lines[k].startswith("."):
            break
        if any(c == f"s_cbranch_execz {t}" for t in refs):
            first = k
            # an if-else: the flow block's own label is the then-branch's skip target
            prev = k - 1
            while prev >= 0 and not code(lines[prev]):
                prev -= 1
            if code(lines[prev]).startswith("s_andn2_saveexec"):
                f = prev
                while f >= 0 and not LABEL.match(lines[f]):
                    f -= 1
                if f >= 0:
                    refs.append(LABEL.match(lines[f]).group(1))
    for k in range(first, -1, -1):
        if "s_and_saveexec" in code(lines[k]):
            return k
    return 0


def code(line):
    return line.split(";")[0].strip()


def scan(path):
    lines = open(path).read().splitlines()
    labels = {}
    for i, ln in enumerate(lines):
        m = LABEL.match(ln)
        if m:
            labels[m.group(1)] = i
    skipped = {c.split()[1] for c in map(code, lines) if c.startswith("s_cbranch_execz ")}
    hits = []
    func = "?"
    for i, ln in enumerate(lines):
        fm = FUNC.match(ln)
        if fm and not ln.startswith("."):
            func = fm.group(1)
        lm = LABEL.match(ln)
        if not lm or lm.group(1) not in skipped:
            continue  # only joins that a skipped branch jumps to (s_cbranch_execz)
        # the join block's prologue: instructions up to the exec restore
        pre, j = [], i + 1
        while j < len(lines):
            s = code(lines[j])
            if not s:
                j += 1
                continue
            if RESTORE.match(s):
                break
            if LABEL.match(lines[j]) or s.startswith(("s_cbranch", "s_branch", "s_endpgm")) or "exec" in s:
                j = -1
                break
            pre.append((j, s))
            j += 1
        if j < 0 or j >= len(lines) or not pre:
            continue
        restore = j
        # live-range split copies: a register copy of a value defined before the region
        # (its source is not written inside the region) must reach every lane of it
        start = region_start(lines, i, lm.group(1))
        inside = set()
        for u in range(start, i):
            s_u = code(lines[u])
            if s_u:
                inside |= decode(s_u)[1]
        written = set()
        for _, s in pre:
            mn, w, r = decode(s)
            if mn.startswith(COPY) and not (r & inside):
                written |= w
        if not written:
            continue
        # the then-branch: the region skipped by `s_cbranch_execz <flow>` whose flow block
        # jumps here (`s_cbranch_execz <this label>` after s_andn2_saveexec)
        then_w = set()
        target = lm.group(1)
        for k in range(i - 1, -1, -1):
            if code(lines[k]) == f"s_cbranch_execz {target}":
                flow = k
                while flow >= 0 and not LABEL.match(lines[flow]):
                    flow -= 1
                if flow < 0:
                    break
                flab = LABEL.match(lines[flow]).group(1)
                for t in range(flow - 1, -1, -1):
                    if code(lines[t]) == f"s_cbranch_execz {flab}":
                        for u in range(t + 1, flow):
                            then_w |= decode(code(lines[u]))[1] if code(lines[u]) else set()
                        break
                break
            if FUNC.match(lines[k]) and not lines[k].startswith("."):
                break
        cand = written - then_w
        if not cand:
            continue
        # read after the restore before a rewrite?
        live = set()
        pending = set(cand)
        for k in range(restore + 1, len(lines)):
            s = code(lines[k])
            if not s:
                continue
            if LABEL.match(lines[k]) or s.startswith(("s_cbranch", "s_branch", "s_endpgm", "s_setpc")):
                live |= pending  # conservative at the end of the straight-line run
                break
            _, w, r = decode(s)
            live |= (r & pending)
            pending -= w
            pending -= live
            if not pending:
                break
        if live:
            hits.append((func, target, restore + 1, sorted(live), pre))
    return hits


def scan_all(paths):
    return [h for p in paths for h in scan(p)]


def main(paths):
    bad = 0
    for p in paths:
        for func, label, line, live, pre in scan(p):
            bad += 1
            print(f"{p}: {func} {label}: exec restored at line {line}; "
                  f"v{live} written before it, read after it, not written by the other branch")
            for ln, s in pre[:8]:
                print(f"    {ln + 1}: {s}")
    print(f"{bad} suspicious join-block placement(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
