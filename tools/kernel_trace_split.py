"""Per-kernel durations in dispatch order from a rocprofv3 kernel_trace.csv, split into
consecutive phases: python tools/kernel_trace_split.py TRACE.csv KERNEL_SUBSTR n1 n2 ...
prints, for each phase of n_i consecutive dispatches of the matching kernel, the mean / min (us)."""
import csv
import sys


def main():
    path, sub = sys.argv[1], sys.argv[2]
    sizes = [int(x) for x in sys.argv[3:]]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if sub in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows.sort()
    d = [x[1] / 1000.0 for x in rows]
    i = 0
    for n in sizes:
        seg = d[i:i + n]
        i += n
        if seg:
            print(f"{sub[:40]:40s} n={len(seg):3d} mean={sum(seg) / len(seg):8.2f} min={min(seg):8.2f} us")
    print(f"total dispatches {len(d)}")


if __name__ == "__main__":
    main()
