set -o pipefail
# Round 5: per-kernel times of the explicit-Schur solve at the cfg5 final-model size.
OUT=gpurun_out/q6f; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tests/perf/ba_schur_time.py 500 258000 0 > $OUT/run.log 2>&1 || { tail -20 $OUT/run.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
tail -5 $OUT/run.log
python3 - <<'PY'
import csv
rows = []
for r in csv.DictReader(open("gpurun_out/q6f/kernel_stats.csv")):
    n = r["Name"].replace("(anonymous namespace)::", "").split("(")[0][:60]
    rows.append((float(r["TotalDurationNs"]) / 1e6, int(r["Calls"]), float(r["AverageNs"]) / 1e3, n))
rows.sort(reverse=True)
for t, c, a, n in rows[:30]:
    print(f"{t:9.2f} ms {c:6d} {a:9.1f} us  {n}")
PY
