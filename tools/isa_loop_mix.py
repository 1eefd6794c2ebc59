"""Instruction mix of a kernel's loop in device assembly (hipcc --cuda-device-only -S).

usage: python tools/isa_loop_mix.py <file.s> <kernel-symbol-substring> [loop-header-label]
Without a header label, lists the kernel's loops (header, depth, blocks, instructions).
With one, prints the opcode mix of every basic block inside that loop (all depths) and the
totals: VALU / SALU / LDS / VMEM / SMEM / waitcnt / branch."""
import collections
import re
import sys


def kernel_body(path, sym):
    s = open(path).read()
    names = [n for n in re.findall(r"^([A-Za-z_]\S*):", s, re.M) if sym in n]
    if not names:
        sys.exit(f"no kernel matching {sym}")
    a = s.index(names[0] + ":")
    b = s.index(".Lfunc_end", a)
    return names[0], s[a:b].split("\n")


def blocks(lines):
    cur, out = "entry", collections.OrderedDict()
    out[cur] = {"loop": None, "ins": []}
    for l in lines[1:]:
        t = l.strip()
        m = re.match(r"^(\.LBB\S+|; %bb\.\d+):?(.*)$", t)
        if m:
            cur = m.group(1).rstrip(":")
            lp = re.search(r"in Loop: Header=(\S+) Depth=(\d+)", t)
            out[cur] = {"loop": (lp.group(1), int(lp.group(2))) if lp else None, "ins": []}
            continue
        if not t or t.startswith((".", ";")):
            continue
        out[cur]["ins"].append(t.split()[0])
    return out


def cat(op):
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith(("global_", "buffer_", "scratch_", "flat_")):
        return "VMEM"
    if op.startswith(("s_load", "s_buffer_load", "s_store")):
        return "SMEM"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "SALU"
    if op.startswith("v_"):
        return "VALU"
    return "other"


def main():
    name, lines = kernel_body(sys.argv[1], sys.argv[2])
    bl = blocks(lines)
    if len(sys.argv) < 4:
        loops = collections.defaultdict(lambda: [0, 0, 0])
        for b, d in bl.items():
            if d["loop"]:
                h, dep = d["loop"]
                loops[h][0] = max(loops[h][0], dep)
                loops[h][1] += 1
                loops[h][2] += len(d["ins"])
        print(name)
        for h, (dep, nb, ni) in loops.items():
            print(f"{h:16s} depth {dep} blocks {nb:4d} instructions {ni}")
        return
    hdr = sys.argv[3]
    # blocks of the loop: from the header to the last block that names it, plus nested ones
    keys = list(bl)
    hdr = hdr if hdr in keys else ".L" + hdr
    # every block whose innermost loop is this one (the layout may rotate the header to the
    # end), plus the blocks laid out between the header and the last such block (nested loops)
    member = [i for i, k in enumerate(keys) if bl[k]["loop"] and ".L" + bl[k]["loop"][0] in (hdr, ".L" + hdr)]
    i0, i1 = min(member), max(member)
    tot = collections.Counter()
    ops = collections.Counter()
    for k in keys[i0:i1 + 1]:
        for op in bl[k]["ins"]:
            tot[cat(op)] += 1
            ops[op] += 1
    print(name, "loop", hdr, dict(tot), "total", sum(tot.values()))
    for op, c in ops.most_common(40):
        print(f"  {op:28s} {c}")


if __name__ == "__main__":
    main()
