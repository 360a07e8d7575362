set -o pipefail
OUT=gpurun_out/q5z; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tests/perf/ba_schur_struct_time.py > $OUT/struct.log 2>&1 || { tail -20 $OUT/struct.log; exit 1; }
cat $OUT/struct.log | grep -v "^$" | head -45
