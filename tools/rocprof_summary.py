"""Summarise a rocprofv3 kernel-trace result (.db or *_kernel_stats.csv) into a markdown
table: python tools/rocprof_summary.py <result.db|stats.csv> [--out profiles/x.md]"""
import argparse
import csv
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    return [(r[0], int(r[1]), float(r[2]), float(r[3]), float(r[4]))
            for r in c.execute("select name,total_calls,total_duration,average,percentage "
                               "from top_kernels")]


def from_csv(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3,
                         float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--out")
    ap.add_argument("--title", default="rocprofv3 --kernel-trace --stats")
    a = ap.parse_args()
    rows = from_db(a.src) if a.src.endswith(".db") else from_csv(a.src)
    lines = [f"# {a.title}", "", f"source: `{a.src}`", "",
             "| kernel | calls | total us | avg us | % |", "|---|---|---|---|---|"]
    for n, calls, tot, avg, pct in rows:
        lines.append(f"| `{n}` | {calls} | {tot:.1f} | {avg:.1f} | {pct:.2f} |")
    text = "\n".join(lines) + "\n"
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)
    sys.stdout.write(text)


if __name__ == "__main__":
    main()
