"""GPU idle time in a rocprofv3 kernel trace, attributed to the kernel before each gap.

python tools/trace_gaps.py <run_kernel_trace.csv> [name_regex]
Prints: the trace span, the summed kernel time, and per "previous kernel" name the gap count and
total idle time (gaps > 2 us), restricted to kernels matching name_regex when given (gaps are
measured between consecutive matching kernels)."""
import collections
import csv
import re
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"[(<].*", "", n)[-48:]


def main():
    path = sys.argv[1]
    rx = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    rows = []
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name") or r.get("Name") or ""
        if rx and not rx.search(name):
            continue
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    if not rows:
        print("no kernels")
        return
    span = rows[-1][1] - rows[0][0]
    busy = sum(e - s for s, e, _ in rows)
    gaps = collections.defaultdict(lambda: [0, 0.0])
    kt = collections.defaultdict(lambda: [0, 0.0])
    for (s0, e0, n0), (s1, e1, n1) in zip(rows, rows[1:]):
        g = s1 - e0
        if g > 2000:
            k = short(n0)
            gaps[k][0] += 1
            gaps[k][1] += g / 1e3
    for s, e, n in rows:
        k = short(n)
        kt[k][0] += 1
        kt[k][1] += (e - s) / 1e3
    print(f"kernels {len(rows)}  span {span / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  "
          f"idle {(span - busy) / 1e6:.3f} ms")
    print("-- idle after (gaps > 2 us): count, total ms")
    for k, (c, t) in sorted(gaps.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"  {k:50s} {c:7d} {t / 1e3:9.3f}")
    print("-- kernel time: count, total ms")
    for k, (c, t) in sorted(kt.items(), key=lambda kv: -kv[1][1])[:30]:
        print(f"  {k:50s} {c:7d} {t / 1e3:9.3f}")


if __name__ == "__main__":
    main()
