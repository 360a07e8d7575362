"""Prints durations and gaps of consecutive dispatches from a rocprofv3 kernel_trace.csv, starting
at the N-th dispatch of a named kernel: python tools/trace_seq.py TRACE.csv KERNEL N COUNT"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0] for r in rows]
idx = [i for i, n in enumerate(names) if n == sys.argv[2]]
i0 = idx[int(sys.argv[3])]
for i in range(i0, min(len(rows), i0 + int(sys.argv[4]))):
    s, e = int(rows[i]["Start_Timestamp"]), int(rows[i]["End_Timestamp"])
    ps = int(rows[i - 1]["End_Timestamp"])
    print(f"{names[i]:24s} dur {(e - s) / 1000:8.2f} us  gap {(s - ps) / 1000:7.2f} us")
