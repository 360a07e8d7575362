set -o pipefail
# Round 4 closing validation (after the K1 knob cleanup, the ORB cache and the bench barrier): whole GPU suite, smoke(), the default bench line, an 8-rank gloo rehearsal of
# the pair-sharded path on this one GPU (the driver's N = 8 code path), rocprofv3 kernel stats.
OUT=gpurun_out/r6u; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -30
tail -1 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().splitlines()[-1]); s=d['stages']; print(d['value'], d['ms_per_step'], d['roofline']['frac'], s['match_ms'], s['ransac_ms'], d['graph_checksum']); c=d['cfg5']; print(c.get('error'), c.get('value'), c.get('s_per_reconstruction'), c.get('ba_phase_s'))"
timeout -k 10 600 python -u bench.py --gpus 8 --dist-backend gloo --device 0 --steps 1 --warmup 1 --no-fp64 --no-cfg3 --no-cfg5 --no-cpu-baseline > $OUT/bench_n8_gloo.json 2> $OUT/bench_n8_gloo.err || { tail -20 $OUT/bench_n8_gloo.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_n8_gloo.json').read().splitlines()[-1]); print(d['n_gpus'], d['graph_checksum'], d['verified_matches_per_step'], d['distributed']['launcher'], [r['pairs'] for r in d['distributed']['per_rank']])"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cfg5 > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -30 $OUT/bench_prof.err; exit 1; }
find $OUT/prof -name "*kernel_stats.csv"
