"""Generate mhpc_minimal_env_amd/csrc/mhpc_dpp.h: the row-broadcast multiply-add blocks of
the backward sweep (mhpc_bws.hip) as inline-assembly sequences of v_fmac_f{64,32}_dpp with
row_newbcast (gfx950: DPP on a 64-bit VALU op supports row_newbcast only).

  v_fmac_f64_dpp acc, src, m row_newbcast:L   acc += src[lane L of this 16-lane row] * m

One instruction per broadcast multiply-add; the compiler emits v_mov_b64_dpp + v_fmac for
the same source (it does not fold DPP into a 64-bit FMA), twice the issue slots.

A block is a list of accumulators and, per round, one term per accumulator; the rounds are
issued round robin over the accumulators (so one accumulator's chain is spaced by the
block's width: a gfx950 FP64 FMA takes ~2 issue slots of dependent latency, and wide blocks
issue at full rate, tools/ubench/dpp_rate.hip).

Hazard rule (GCNHazardRecognizer::checkDPPHazards, MI300 ISA "manually inserted wait
states"): a DPP instruction may not read a VGPR written in the previous 2 wait states.  The
compiler cannot see inside inline assembly, so every block
  * starts with s_nop 1 (2 wait states: covers whatever the compiler placed before it), and
  * pads with s_nop when it has fewer than 3 accumulators, so that an accumulator is never
    re-read within 2 wait states of its last write.
Sources and multipliers are never written inside a block.  The blocks are volatile: they keep
their source order (the sweep interleaves S and Q column blocks to bound register pressure).
tools/check_dpp_hazards.py checks the shipped assembly for the rule (build gate,
csrc/Makefile).

usage: python tools/gen_dpp_asm.py > mhpc_minimal_env_amd/csrc/mhpc_dpp.h
"""


def lam(nq, i):
    """Lane of matrix row / column i in a 16-lane row (mhpc_bws.hip: Rows<NQ>::lam)."""
    nx = 2 * nq
    if i < nq:
        return 2 * i
    if i < nx:
        return 2 * (i - nq) + 1
    return i if i < 16 else 14 + (i - 16)


class Block:
    """terms[r][a] = (src operand text, m operand text, lane) for accumulator a in round r."""

    def __init__(self, name, naccs, arrays, terms, doc):
        self.name, self.naccs, self.arrays, self.terms, self.doc = name, naccs, arrays, terms, doc

    @staticmethod
    def round_terms(rnd):
        """(accumulator, term) pairs of a round: terms are (src, m, lane) for accumulators
        0, 1, ... in order, or (acc, src, m, lane) for a sparse round."""
        return [(t[0], t[1:]) if len(t) == 4 else (a, t) for a, t in enumerate(rnd)]

    def emit(self):
        # operand numbering: accumulators, then every array element used (in order of use)
        ops, index = [], {}
        nxt = self.naccs
        for rnd in self.terms:
            for _, (src, m, _) in self.round_terms(rnd):
                for e in (src, m):
                    if e not in index:
                        index[e] = nxt
                        ops.append(e)
                        nxt += 1
        assert nxt <= 30, (self.name, nxt)
        out = [f"// {self.doc}",
               "template <class T>",
               f"__device__ __forceinline__ void {self.name}("
               + ", ".join(f"T& a{a}" for a in range(self.naccs)) + ", "
               + ", ".join(f"const T* {n}" for n in self.arrays) + ") {"]
        for t, mn in (("double", "v_fmac_f64_dpp"), ("float", "v_fmac_f32_dpp")):
            lines = ["s_nop 1"]
            k = 0
            last = {}  # accumulator -> issue slot of its last write
            for rnd in self.terms:
                for a, (src, m, lane) in self.round_terms(rnd):
                    # an accumulator re-read within 2 wait states of its write: pad
                    gap = k - last[a] - 1 if a in last else 2
                    if gap < 2:
                        lines.append(f"s_nop {1 - gap}")
                        k += 2 - gap
                    lines.append(f"{mn} %{a}, %{index[src]}, %{index[m]} row_newbcast:{lane} "
                                 "row_mask:0xf bank_mask:0xf")
                    last[a] = k
                    k += 1
            kw = "if constexpr (sizeof(T) == 8)" if t == "double" else "else"
            out.append(f"  {kw}")
            out.append('    asm volatile("' + "\\n\\t".join(lines) + '"')
            out.append("        : " + ", ".join(f'"+v"(a{a})' for a in range(self.naccs)))
            out.append("        : " + ", ".join(f'"v"({e})' for e in ops) + ");")
        out.append("}")
        return "\n".join(out)


def col_block(name, nq, cols, r, arrays, src_of, m_of, doc):
    """acc c += sum_r bcast(src_of(c, r), lam(c)) * m_of(c, r): broadcast lane per column."""
    terms = [[(src_of(c, j), m_of(c, j), lam(nq, c)) for c in cols] for j in range(r)]
    return Block(name, len(cols), arrays, terms, doc)


def lane_block(name, lanes, c, arrays, doc):
    """acc a += sum_r bcast(s_a, lanes[r]) * m[r]: one broadcast source per accumulator."""
    terms = [[(f"s[{a}]", f"m[{j}]", lanes[j]) for a in range(c)] for j in range(len(lanes))]
    return Block(name, c, arrays, terms, doc)


def blocks():
    B = []
    # ---- whole body (NQ = 7) ----
    # S = H [A B]: S[c] += sum_r bcast(W[r], lam(c)) * H[7 + r]; columns 16, 17 from W2
    for nm, cols in (("a", range(0, 6)), ("b", range(6, 12)), ("c", range(12, 18))):
        B.append(col_block(
            f"wb_s_{nm}", 7, list(cols), 7, ["w1", "w2", "h"],
            lambda c, j: f"w1[{j}]" if c < 16 else f"w2[{j}]", lambda c, j: f"h[{j}]",
            f"whole body S = H [A B], columns {cols.start}..{cols.stop - 1}"))
    # stance rank-2 terms: Q[.][d] += sum_z bcast(G2[z], lam(d)) * cc[z]
    for nm, cols in (("a", range(0, 6)), ("b", range(6, 12))):
        B.append(col_block(f"wb_st_{nm}", 7, list(cols), 2, ["g", "cc"],
                           lambda c, j: f"g[{j}]", lambda c, j: f"cc[{j}]",
                           f"whole body C'lyyC / D'lyyC terms, columns {cols.start}..{cols.stop - 1}"))
    # columns 12..17 and the second control set (rows 16, 17: only columns 16, 17)
    terms = []
    for j in range(2):
        rnd = [(f"g[{j}]", f"cc[{j}]", lam(7, c)) for c in range(12, 16)]
        rnd += [(f"g2[{j}]", f"cc[{j}]", lam(7, c)) for c in (16, 17)]
        rnd += [(f"g2[{j}]", f"cc2[{j}]", lam(7, c)) for c in (16, 17)]
        terms.append(rnd)
    B.append(Block("wb_st_c", 8, ["g", "g2", "cc", "cc2"], terms,
                   "whole body stance terms, columns 12..17 (6 accumulators) and the control rows 2, 3"
                   " (2 accumulators)"))
    # H update: H[rho][j] += sum_a bcast(Qxu[a], lam(j)) * K[a]
    for nm, cols in (("a", range(0, 7)), ("b", range(7, 14))):
        B.append(col_block(f"wb_h_{nm}", 7, list(cols), 4, ["qxu", "k"],
                           lambda c, j: f"qxu[{j}]", lambda c, j: f"k[{j}]",
                           f"whole body H update, columns {cols.start}..{cols.stop - 1}"))
    # impact step H = T Px: H[i][j] += sum_m bcast(Pc[m], lam(j)) * T[m] (m in one half)
    for nm, cols in (("a", range(0, 7)), ("b", range(7, 14))):
        B.append(col_block(f"wb_p_{nm}", 7, list(cols), 7, ["pc", "t"],
                           lambda c, j: f"pc[{j}]", lambda c, j: f"t[{j}]",
                           f"impact step H = T Px, columns {cols.start}..{cols.stop - 1}, seven m"))
    # Q = [A B]' S, G column, Px' H2: one broadcast source per accumulator, lanes 2r+1 / 2r
    odd7, even7 = [1, 3, 5, 7, 9, 11, 13], [0, 2, 4, 6, 8, 10, 12]
    for c in (3, 6, 7, 8):
        B.append(lane_block(f"sb_odd7_{c}", odd7, c, ["s", "m"],
                            f"acc a += sum_r bcast(s[a], 2r + 1) * m[r], r < 7, {c} accumulators"))
    for c in (7, 8):
        B.append(lane_block(f"sb_even7_{c}", even7, c, ["s", "m"],
                            f"acc a += sum_r bcast(s[a], 2r) * m[r], r < 7, {c} accumulators"))
    # ---- whole body, two rows per problem (sweep_wb2): row A holds the configuration
    # columns 0..6, row B the velocity columns 7..13 in the same slots (its broadcast set puts
    # column 7 + s on lane 2 s), both the control columns 14..17 ----
    terms = []
    for j in range(7):
        rnd = [(f"wb[{j}]", f"h[{j}]", 12), (f"wb[{j}]", f"h[{j}]", 14), (f"wb[{j}]", f"h[{j}]", 15),
               (f"w2[{j}]", f"h[{j}]", 14), (f"w2[{j}]", f"h[{j}]", 15)]
        terms.append(rnd)
    B.append(Block("wb2_s_b", 5, ["wb", "w2", "h"], terms,
                   "two-row S = H [A B], slots 6..10 (column 6 / 13, 14, 15, 16, 17)"))
    terms = []
    for j in range(2):
        rnd = [(f"g[{j}]", f"cc[{j}]", 12), (f"g[{j}]", f"cc[{j}]", 14), (f"g[{j}]", f"cc[{j}]", 15),
               (f"g2[{j}]", f"cc[{j}]", 14), (f"g2[{j}]", f"cc[{j}]", 15),
               (f"g2[{j}]", f"cc2[{j}]", 14), (f"g2[{j}]", f"cc2[{j}]", 15)]
        terms.append(rnd)
    B.append(Block("wb2_st_b", 7, ["g", "g2", "cc", "cc2"], terms,
                   "two-row stance terms, slots 6..10 and the control rows 2, 3"))
    # ---- SRB (NQ = 3) ----
    # sparse S = H [A B] of the SRB knot: the terms whose W entry is structurally non-zero
    # (FBDynamics_par.c: row 3 has columns 3, 6, 8; row 4 columns 4, 7, 9; row 5 columns 0, 1,
    # 5..9), in the dense blocks' order r = 0, 1, 2 -- a skipped term added an exact zero
    nzr = {0: [2], 1: [2], 2: [], 3: [0], 4: [1], 5: [2], 6: [0, 2], 7: [1, 2], 8: [0, 2], 9: [1, 2]}
    for nm, cols in (("a", [0, 1, 3, 4]), ("b", [5, 6, 7, 8, 9])):
        rounds = []
        for j in range(2):
            rnd = [(a, f"w[{nzr[c][j]}]", f"h[{nzr[c][j]}]", lam(3, c))
                   for a, c in enumerate(cols) if j < len(nzr[c])]
            if rnd:
                rounds.append(rnd)
        B.append(Block(f"srb_sp_{nm}", len(cols), ["w", "h"], rounds,
                       f"SRB S = H [A B], structurally non-zero terms of columns {cols}"))
    B.append(col_block("srb_h", 3, list(range(6)), 4, ["qxu", "k"],
                       lambda c, j: f"qxu[{j}]", lambda c, j: f"k[{j}]", "SRB H update"))
    for c in (5, 6):
        B.append(lane_block(f"sb_odd3_{c}", [1, 3, 5], c, ["s", "m"],
                            f"acc a += sum_r bcast(s[a], 2r + 1) * m[r], r < 3, {c} accumulators"))
    return B


def main():
    print("// GENERATED by tools/gen_dpp_asm.py -- do not edit.  Row-broadcast multiply-add")
    print("// blocks of the backward sweep (v_fmac_f{64,32}_dpp row_newbcast); the hazard rule they")
    print("// keep is in the generator's docstring, tools/check_dpp_hazards.py checks the build.")
    print("#pragma once")
    print("#include <hip/hip_runtime.h>")
    print()
    print("namespace MHPC_NS {")
    print()
    for b in blocks():
        print(b.emit())
        print()
    print("}  // namespace MHPC_NS")


if __name__ == "__main__":
    main()
