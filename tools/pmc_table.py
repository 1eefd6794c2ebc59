"""Per-kernel sums of every counter collected under a rocprofv3 --pmc output tree:
python tools/pmc_table.py <dir>"""
import collections
import csv
import glob
import sys

tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for path in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    with open(path) as f:
        for r in csv.DictReader(f):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add((path, r["Dispatch_Id"]))
for k in sorted(tot):
    print(k, "dispatches", len(disp[k]))
    for c, v in sorted(tot[k].items()):
        print(f"   {c:32s} {v:16.0f}")
