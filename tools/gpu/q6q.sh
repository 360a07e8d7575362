set -o pipefail
# Round 5: kernel totals of one cfg5 reconstruction with the explicit Schur system (bench --config cfg5).
OUT=gpurun_out/q6q; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/run.log 2>&1 || { tail -20 $OUT/run.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
python3 - <<'PY'
import csv
rows = []
for r in csv.DictReader(open("gpurun_out/q6q/kernel_stats.csv")):
    n = r["Name"].replace("(anonymous namespace)::", "").split("(")[0][:50]
    rows.append((float(r["TotalDurationNs"]) / 1e6, int(r["Calls"]), n))
rows.sort(reverse=True)
tot = sum(r[0] for r in rows)
print("total_ms (2 reconstructions + side measurements)", round(tot, 1))
for t, c, n in rows[:30]:
    print(f"{t:9.2f} ms {c:6d}  {n}")
PY
