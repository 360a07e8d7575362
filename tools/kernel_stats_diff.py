"""Per-kernel total-time difference of two rocprofv3 kernel_stats.csv files (B - A), largest first.
Usage: python tools/kernel_stats_diff.py A.csv B.csv [N]"""
import csv
import sys


def load(p):
    d = {}
    for r in csv.DictReader(open(p)):
        n = r["Name"].replace("(anonymous namespace)::", "").split("(")[0][:60]
        c, t = d.get(n, (0, 0.0))
        d[n] = (c + int(r["Calls"]), t + int(r["TotalDurationNs"]) / 1e6)
    return d


def main():
    a, b = load(sys.argv[1]), load(sys.argv[2])
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    rows = sorted(((b.get(k, (0, 0.0))[1] - a.get(k, (0, 0.0))[1], k) for k in set(a) | set(b)),
                  reverse=True)
    print("delta_ms  kernel  calls_a ms_a  calls_b ms_b")
    for dt, k in rows[:n] + rows[-5:]:
        ca, ta = a.get(k, (0, 0.0))
        cb, tb = b.get(k, (0, 0.0))
        print(f"{dt:8.2f} {k:60s} {ca:6d} {ta:8.2f} {cb:6d} {tb:8.2f}")
    print("total_ms", round(sum(t for _, t in a.values()), 2), round(sum(t for _, t in b.values()), 2))


if __name__ == "__main__":
    main()
