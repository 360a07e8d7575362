set -o pipefail
# Round 5: where the chunk mode's cfg5 overhead sits — BAProblem set-up pieces, then kernel traces
# of cfg5 with SFM_BA_CHUNKS=0 and 8 (per-kernel totals compared).
OUT=gpurun_out/q5m; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u tests/perf/ba_setup_time.py > $OUT/setup.json 2> $OUT/setup.err || { tail -20 $OUT/setup.err; exit 1; }
cat $OUT/setup.json
for c in 0 8; do
  SFM_BA_CHUNKS=$c timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_c$c -o run --output-format csv -- python3 bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/c$c.log 2>&1 || { tail -20 $OUT/c$c.log; exit 1; }
  find $OUT/prof_c$c -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/stats_c$c.csv
done
python3 - <<'PY'
import csv
def load(p):
    d = {}
    for r in csv.DictReader(open(p)):
        n = r["Name"].split("(")[0].replace("(anonymous namespace)::", "")[:60]
        d[n] = (int(r["Calls"]), int(r["TotalDurationNs"]) / 1e6)
    return d
a, b = load("gpurun_out/q5m/stats_c0.csv"), load("gpurun_out/q5m/stats_c8.csv")
rows = []
for n in set(a) | set(b):
    ca, ta = a.get(n, (0, 0.0)); cb, tb = b.get(n, (0, 0.0))
    rows.append((tb - ta, n, ca, ta, cb, tb))
rows.sort(reverse=True)
print("delta_ms kernel calls0 ms0 calls8 ms8")
for r in rows[:25]:
    print(f"{r[0]:8.2f} {r[1]:60s} {r[2]:6d} {r[3]:8.2f} {r[4]:6d} {r[5]:8.2f}")
print("total", sum(t for _, t in a.values()), sum(t for _, t in b.values()))
PY
