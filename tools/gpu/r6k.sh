set -o pipefail
# Round 4: RANSAC_PV = 128 default — the whole GPU suite, the default bench line, and a
# rocprofv3 kernel-trace summary of the same bench command.
OUT=gpurun_out/r6k; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -30
tail -2 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['stages']['ransac_ms'], d['graph_checksum']); c=d['cfg5']; print(c.get('error'), c.get('value'), c.get('s_per_reconstruction'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --no-cfg5 > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -30 $OUT/bench_prof.err; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -3
