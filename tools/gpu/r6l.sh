set -o pipefail
# Round 4: K1 / K2 overlap A/B at cfg4: the parity test of GraphBuilder.run_overlapped, the
# standalone A/B (tests/perf/overlap_ab.py), then bench.py --pieces 1 / 2 / 4 interleaved.
OUT=gpurun_out/r6l; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python -u tests/perf/overlap_stats_probe.py > $OUT/stats_probe.txt 2>&1 || { tail -30 $OUT/stats_probe.txt; exit 1; }
cat $OUT/stats_probe.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_host.py -k overlapped -v -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_overlap.log 2>&1
rc=$?
grep -E "^E  |FAILED|passed|failed" $OUT/pytest_overlap.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u tests/perf/overlap_ab.py 500 4096 2 > $OUT/overlap.jsonl 2> $OUT/overlap.err || { tail -30 $OUT/overlap.err; exit 1; }
cat $OUT/overlap.jsonl
for r in 1 2; do
  for p in 1 2 4; do
    timeout -k 10 300 python -u bench.py --no-cfg5 --no-cfg3 --no-fp64 --no-cpu-baseline --pieces $p > $OUT/bench_p$p.$r.json 2> $OUT/bench_p$p.$r.err || { tail -30 $OUT/bench_p$p.$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/bench_p$p.$r.json').read().splitlines()[-1]); s=d['stages']; print('pieces', $p, 'round', $r, round(d['ms_per_step'],2), round(s['match_ms'],2), round(s['ransac_ms'],2), round(s['k1_k2_span_ms'],2), d['graph_checksum'])"
  done
done
