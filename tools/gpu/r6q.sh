set -o pipefail
# Round 4: full-size cross-implementation agreement at cfg4 (tests/perf/cfg4_cross_impl.py).
OUT=gpurun_out/r6q; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u tests/perf/cfg4_cross_impl.py > $OUT/cross.json 2> $OUT/cross.err || { tail -30 $OUT/cross.err; exit 1; }
cat $OUT/cross.json
