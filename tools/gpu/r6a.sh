set -o pipefail
# Round 4, first call: cfg5 scene probes (bench.py --config cfg5 at two scene-point counts), the
# whole GPU suite (no -x: test failures do not stop the call; a crash or time limit does), the
# ordered-pair timing, then the default bench line (cfg4 + cfg3 / cfg5 side legs).
OUT=gpurun_out/r6a; mkdir -p $OUT
export TMPDIR=/tmp
for np in 100000 300000; do
  timeout -k 10 300 python -u bench.py --config cfg5 --n-pts $np --steps 1 --warmup 1 > $OUT/cfg5_$np.json 2> $OUT/cfg5_$np.err || { tail -30 $OUT/cfg5_$np.err; exit 1; }
  echo "cfg5 n_pts=$np: $(python3 -c "import json,sys; d=json.loads(open('$OUT/cfg5_$np.json').read().splitlines()[-1]); c=d['cfg5']; print(d['value'], c['s_per_reconstruction'], c['registered'], c['points'], c['observations'], c['median_reproj_px'], c['lm_steps'], c['cg_iters'], c['stage_s'])")"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -30
tail -2 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tests/perf/ordered_pairs_time.py > $OUT/ordered_pairs.json 2> $OUT/ordered_pairs.err && cat $OUT/ordered_pairs.json &&
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('cfg5'))"
