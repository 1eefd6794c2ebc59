"""Build gate: DPP read-after-write hazards in device assembly (hipcc --cuda-device-only -S).

gfx9 rule (MI300/MI355X ISA "manually inserted wait states"; LLVM
GCNHazardRecognizer::checkDPPHazards): a DPP instruction may not read a VGPR written by any
instruction in the previous 2 wait states, nor follow a VALU write of EXEC within 5.  The
compiler enforces this for the DPP instructions it emits; the sweep's row-broadcast
multiply-adds (mhpc_dpp.h) are inline assembly, which the compiler cannot look into.  This
scan replays every function linearly: each instruction is one wait state, s_nop N is N+1; at a
label the predecessor is unknown, so an inline-assembly DPP instruction (v_fmac_*_dpp) within
2 wait states of a label is reported unless an s_nop covers it (every generated block starts
with s_nop 1).  Compiler-emitted DPP moves are checked within straight-line code only.

usage: python tools/check_dpp_hazards.py <file.s> [...]    exit 1 on any hazard
"""
import re
import sys

REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")
NO_DEST = ("global_store", "buffer_store", "scratch_store", "flat_store", "ds_write", "ds_store",
           "s_", "global_atomic", "buffer_atomic", "ds_add", "v_cmp_", "v_cmpx_", "v_readlane",
           "v_readfirstlane", "exp ", "v_nop")


def regs(text):
    out = set()
    for kind, lo, hi, one in REG.findall(text):
        if one:
            out.add((kind, int(one)))
        else:
            out.update((kind, r) for r in range(int(lo), int(hi) + 1))
    return out


def split_ops(ins):
    parts = ins.split(None, 1)
    op = parts[0]
    ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
    return op, ops


def check(path):
    bad = []
    fn = None
    hist = []  # (wait states elapsed when written, set of regs); newest last
    t = 0      # wait-state clock
    label_t = -10
    exec_valu_t = -10
    with open(path) as f:
        for ln, raw in enumerate(f, 1):
            line = raw.split(";")[0].rstrip()
            s = line.strip()
            if not s:
                continue
            m = re.match(r"^([A-Za-z_.$][\w.$]*):", s)
            if m:
                if not s.startswith("."):
                    fn = m.group(1)
                label_t = t
                hist = []
                continue
            if s.startswith("."):
                continue
            op, ops = split_ops(s)
            if op == "s_nop":
                t += int(ops[0], 0) + 1
                continue
            if "_dpp" in op:
                reads = set()
                src = ops[1:] if not op.startswith(("v_fmac", "v_mac")) else ops
                for o in src:
                    if o.startswith(("v", "a")) and not o.startswith(("vcc",)):
                        reads |= regs(o)
                for wt, ws in hist:
                    if t - wt - 1 < 2 and ws & reads:
                        bad.append(f"{path}:{ln}: {fn}: {s}  (operand written {t - wt - 1} "
                                   "wait state(s) earlier)")
                        break
                if op.startswith("v_fmac") and t - label_t < 2:
                    bad.append(f"{path}:{ln}: {fn}: {s}  (within 2 wait states of a label)")
                if t - exec_valu_t - 1 < 5:
                    bad.append(f"{path}:{ln}: {fn}: {s}  (VALU write of EXEC within 5)")
            # record the write of this instruction
            if ops and not op.startswith(NO_DEST) and (ops[0].startswith("v") or ops[0].startswith("a")):
                w = regs(ops[0])
                if w:
                    hist.append((t, w))
                    hist = hist[-8:]
            if op.startswith("v_cmpx_") or (op.startswith("v_") and ops and ops[0].startswith("exec")):
                exec_valu_t = t
            t += 1
    return bad


def main(paths):
    bad = []
    n = 0
    for p in paths:
        bad += check(p)
        n += 1
    for b in bad:
        print(b)
    print(f"check_dpp_hazards: {n} file(s), {len(bad)} hazard(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
