set -o pipefail
# Round 4: cfg5 with the bundle adjustments' phase times (selection / setup / LM / post / total),
# after the device-side reprojection filter; the incremental GPU tests.
OUT=gpurun_out/r6m; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_incremental.py -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_inc.log 2>&1 || { grep -E "^E  |FAILED" $OUT/pytest_inc.log | head; tail -3 $OUT/pytest_inc.log; exit 1; }
tail -1 $OUT/pytest_inc.log
timeout -k 10 300 python -u bench.py --config cfg5 --steps 3 --warmup 1 > $OUT/cfg5.json 2> $OUT/cfg5.err || { tail -30 $OUT/cfg5.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/cfg5.json').read().splitlines()[-1]); c=d['cfg5']; print(d['value'], d['ms_per_step']); print({k: c.get(k) for k in ('registered','points','observations','median_reproj_px','lm_steps','cg_iters','stage_s','ba_phase_s')})"
