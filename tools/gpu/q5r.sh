set -o pipefail
# Round 5: per-kernel durations of the CG iteration at the cfg5 final-model size.
OUT=gpurun_out/q5r; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tests/perf/ba_solve_bench.py 500 258000 4 > $OUT/run.log 2>&1 || { tail -20 $OUT/run.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/q5r/kernel_stats.csv")):
    n = r["Name"].replace("(anonymous namespace)::", "").split("(")[0]
    if n.startswith(("bas_", "ba_")):
        print(f'{n:28s} calls={r["Calls"]:>6s} avg_us={float(r["AverageNs"])/1000:8.2f} min_us={float(r["MinNs"])/1000:8.2f}')
PY
