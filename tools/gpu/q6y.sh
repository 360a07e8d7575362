set -o pipefail
# Round 5 validation: whole GPU suite, smoke(), the default bench line (cfg4 + cfg4_local / cfg3 /
# cfg5 legs), rocprofv3 kernel stats of the bench (no cfg5 leg).
OUT=gpurun_out/q6y; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -30
tail -1 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
OUT=gpurun_out/q6y; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_ransac.py::test_ransac_stats_identity > $OUT/pytest_stats.log 2>&1 || { tail -30 $OUT/pytest_stats.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().splitlines()[-1]); s=d['stages']; print(d['value'], d['ms_per_step'], d['roofline']['frac'], s['match_ms'], s['ransac_ms'], d['graph_checksum']); l=d.get('cfg4_local', {}); print('local', l.get('error'), l.get('value'), l.get('verified_pairs'), l.get('match_ms'), l.get('ransac_ms')); c=d['cfg5']; print('cfg5', c.get('error'), c.get('value'), c.get('s_per_reconstruction'), c.get('ba_phase_s')); print('cfg3', d['cfg3']['match_ms'], d['cfg3']['k1_roofline']['frac'])"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cfg5 --no-local > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -30 $OUT/bench_prof.err; exit 1; }
find $OUT/prof -name "*kernel_stats.csv"
