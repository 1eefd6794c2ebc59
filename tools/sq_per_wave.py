"""Per-wave view of tools/gpu_pmc_stalls.sh output (pmc_table format): instructions per wave
by type, wave cycles (SQ cycle counters count 4-cycle quads) and the share of wave cycles
waiting / issuing.  usage: python tools/sq_per_wave.py <sq_*.txt>"""
import re
import sys

txt = open(sys.argv[1]).read()
for b in re.split(r"\n(?=\S)", txt):
    lines = b.strip().split("\n")
    if not lines or "dispatches" not in lines[0]:
        continue
    d = {}
    for l in lines[1:]:
        p = l.split()
        if len(p) == 2:
            d[p[0]] = float(p[1])
    if "SQ_INSTS_VALU" not in d or not d.get("SQ_WAVES"):
        continue
    w, nd = d["SQ_WAVES"], int(lines[0].split()[-1])
    wc = d["SQ_WAVE_CYCLES"]
    print(f"{lines[0].split(' dispatches')[0][:44]:44s} waves/disp {w / nd:7.0f}  per wave: VALU {d['SQ_INSTS_VALU'] / w:7.0f}"
          f" SALU {d['SQ_INSTS_SALU'] / w:6.0f} LDS {d.get('SQ_INSTS_LDS', 0) / w:5.0f} cycles {4 * wc / w:8.0f}"
          f" | wait_any {d['SQ_WAIT_ANY'] / wc:.2f} wait_inst {d['SQ_WAIT_INST_ANY'] / wc:.2f}"
          f" active {d['SQ_ACTIVE_INST_ANY'] / wc:.2f} valu {d['SQ_ACTIVE_INST_VALU'] / wc:.2f}")
