set -o pipefail
# Round 5: per-kernel times of both mutual-rule K1 implementations in one process (rocprofv3).
OUT=gpurun_out/q5f; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tests/perf/k1_grp_ab.py 1 > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); echo $f; head -20 $f | cut -c1-200
