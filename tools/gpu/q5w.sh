set -o pipefail
# Round 5: explicit reduced camera system timings (cfg5-like tracks at the final-model size and a
# uniform 5-observation problem), then a kernel trace of the cfg5-like run.
OUT=gpurun_out/q5w; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tests/perf/ba_schur_time.py > $OUT/grid.json 2> $OUT/grid.err || { tail -20 $OUT/grid.err; exit 1; }
grep '^{' $OUT/grid.json
timeout -k 10 300 python -u tests/perf/ba_schur_time.py 500 100000 5 > $OUT/u5.json 2> $OUT/u5.err || { tail -20 $OUT/u5.err; exit 1; }
grep '^{' $OUT/u5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tests/perf/ba_schur_time.py > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/q5w/kernel_stats.csv")):
    n = r["Name"].replace("(anonymous namespace)::", "").split("(")[0]
    if n.startswith(("bas_", "ba_")) or "sort" in n or "unique" in n:
        print(f'{n[:40]:40s} calls={r["Calls"]:>6s} avg_us={float(r["AverageNs"])/1000:8.2f} min_us={float(r["MinNs"])/1000:8.2f} tot_ms={float(r["TotalDurationNs"])/1e6:8.2f}')
PY
