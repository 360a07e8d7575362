set -o pipefail
# Round 4: K1 / K2 overlap A/B at cfg4 (tests/perf/overlap_ab.py): chunked pair list, K1 chunk i+1
# on one stream while K2 chunk i runs on another (two sfm contexts).
OUT=gpurun_out/r6l; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u tests/perf/overlap_ab.py 500 4096 2 > $OUT/overlap.jsonl 2> $OUT/overlap.err || { tail -30 $OUT/overlap.err; exit 1; }
cat $OUT/overlap.jsonl
