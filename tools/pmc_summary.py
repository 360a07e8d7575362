"""Summarise rocprofv3 counter_collection CSVs: mean per dispatch, per (kernel, counter)."""
import collections
import csv
import glob
import re
import sys

d = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).replace("void ", "")
        d[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
kern = sorted({k for k, _ in d})
for k in kern:
    print(k)
    for (kk, c), v in sorted(d.items()):
        if kk == k:
            print(f"   {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
