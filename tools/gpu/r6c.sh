set -o pipefail
# Round 4: the whole GPU suite (no -x: failures do not stop the call; a crash or time limit
# does), the ordered-pair timing, the default bench line (cfg4 + cfg3 / cfg5 side legs), then
# the K1 prologue A/B (pair-info record vs the pair_order -> pairs -> n_kp chain), interleaved.
OUT=gpurun_out/r6c; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -30
tail -2 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u tests/perf/ordered_pairs_time.py > $OUT/ordered_pairs.json 2> $OUT/ordered_pairs.err && cat $OUT/ordered_pairs.json &&
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac']); c=d.get('cfg5',{}); print({k: c.get(k) for k in ('error','value','s_per_reconstruction','registered','points','observations','median_reproj_px','lm_steps','cg_iters','stage_s','pcg_branches')}); print(c.get('ba_rooflines'))"
K1_ONLY_BENCH_RULE=1 timeout -k 10 300 bash tools/ab_k1.sh 3 base chain > $OUT/k1_ab.txt 2>&1; cat $OUT/k1_ab.txt
