# Round 6: K1 / K2 overlap on two streams with two contexts (tests/perf/k1k2_overlap.py) on the
# cfg4 scene at the bench's 4096 hypotheses: serial vs pipelined.
set -o pipefail
O=gpurun_out/s32; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python tests/perf/k1k2_overlap.py 31250 62500 > $O/overlap.jsonl 2> $O/overlap.err || { tail -20 $O/overlap.err; exit 1; }
cat $O/overlap.jsonl
