"""Loop-invariant registers of a kernel loop in device assembly: the VGPRs / AGPRs a loop
reads but never writes (values hoisted out of it, live through every iteration).

usage: python tools/isa_loop_regs.py <file.s> <kernel-symbol-substring> <loop-header-label>
(loop headers: python tools/isa_loop_mix.py <file.s> <kernel>)"""
import re
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
from isa_loop_mix import kernel_body  # noqa: E402

# opcodes whose first operand is read, not written
NO_DEF = ("ds_write", "global_store", "buffer_store", "scratch_store", "flat_store", "s_cmp",
          "s_waitcnt", "s_barrier", "s_cbranch", "s_branch", "s_nop", "s_setprio", "s_store")


def regs(op):
    out = []
    for m in re.finditer(r"\b([vsa])\[(\d+):(\d+)\]|\b([vsa])(\d+)\b", op):
        if m.group(1):
            out += [m.group(1) + str(i) for i in range(int(m.group(2)), int(m.group(3)) + 1)]
        else:
            out.append(m.group(4) + m.group(5))
    return out


def main():
    name, lines = kernel_body(sys.argv[1], sys.argv[2])
    hdr = sys.argv[3].lstrip(".L")
    cur, loop_of, body = None, {}, {}
    order = []
    for l in lines[1:]:
        t = l.strip()
        m = re.match(r"^(\.LBB\S+|; %bb\.\d+):?(.*)$", t)
        if m:
            cur = m.group(1).rstrip(":")
            lp = re.search(r"Loop: Header=(\S+) Depth=(\d+)", t)
            loop_of[cur] = lp.group(1) if lp else None
            body[cur] = []
            order.append(cur)
            continue
        if cur and t and not t.startswith((".", ";")):
            body[cur].append(t)
    i0 = order.index(".L" + hdr)
    i1 = max(i for i, k in enumerate(order) if loop_of.get(k) == hdr)
    w, r, n = set(), set(), 0
    for k in order[i0:i1 + 1]:
        for t in body[k]:
            n += 1
            parts = t.split(None, 1)
            if len(parts) < 2:
                continue
            ops = [o.strip() for o in parts[1].split(",")]
            if parts[0].startswith(NO_DEF):
                for o in ops:
                    r.update(regs(o))
            else:
                w.update(regs(ops[0]))
                for o in ops[1:]:
                    r.update(regs(o))
    print(name, "loop", hdr, "instructions", n)
    for k in "vas":
        inv = sorted((x for x in r - w if x[0] == k), key=lambda x: int(x[1:]))
        wr = [x for x in w if x[0] == k]
        print(f"{k}: written {len(wr)}, read-only (loop-invariant) {len(inv)}")
        if k != "s":
            print("  " + " ".join(inv))


if __name__ == "__main__":
    main()
