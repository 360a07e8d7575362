set -o pipefail
# Round 5: cfg2 (BASELINE configs[1]: 50 x 2048, L2 + fused ratio test, no cross check) — the
# ratio path against the mutual kernel: call times, then one PMC pass (MFMA busy, instructions).
OUT=gpurun_out/q6w; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u tests/perf/k1_cfg2_time.py > $OUT/time.log 2>&1 || { tail -20 $OUT/time.log; exit 1; }
grep rule $OUT/time.log
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 tests/perf/k1_cfg2_time.py > $OUT/kt.log 2>&1 || { tail -5 $OUT/kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "l2fr_scan_kernel|mfma_mutual_kernel|l2fr_recover_kernel" -d $OUT/p1 -o run --output-format csv -- python3 tests/perf/k1_cfg2_time.py > $OUT/p1.log 2>&1 || { tail -5 $OUT/p1.log; exit 1; }
python3 tools/pmc_summary.py $OUT/p1 > $OUT/summary.txt && cat $OUT/summary.txt
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/q6w/kt/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].replace("(anonymous namespace)::", "").split("(")[0]
    if "l2fr" in n or "mutual" in n:
        print(f"{n[:50]:50s} calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1e3:9.1f} us")
PY
