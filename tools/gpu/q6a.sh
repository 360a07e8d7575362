set -o pipefail
OUT=gpurun_out/q6a; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tests/perf/ba_solve_bench.py 500 258000 4 > $OUT/ba_solve_258k.json 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
grep '^{' $OUT/ba_solve_258k.json | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('cg', d['cg_iter_ms'], 'setup_backsub', d['setup_backsub_ms'], 'chunked', d['chunked'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tests/perf/ba_solve_bench.py 500 258000 4 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/q6a/kernel_stats.csv")):
    n = r["Name"].replace("(anonymous namespace)::", "").split("(")[0]
    if "camera_setup" in n or "camera_finish" in n or "point_setup" in n or "bas_soa" in n:
        print(f'{n:28s} calls={r["Calls"]:>6s} avg_us={float(r["AverageNs"])/1000:8.2f} min_us={float(r["MinNs"])/1000:8.2f}')
PY
