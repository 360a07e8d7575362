set -o pipefail
# Round 4: the whole GPU suite, the default bench line (cfg4 + cfg3 / cfg5 legs) and the cfg5 line
# after the device-side observation selection of the incremental driver's bundle adjustments.
OUT=gpurun_out/r6h; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -30
tail -2 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --config cfg5 --steps 3 --warmup 1 > $OUT/cfg5.json 2> $OUT/cfg5.err || { tail -30 $OUT/cfg5.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/cfg5.json').read().splitlines()[-1]); c=d['cfg5']; print(d['value'], d['ms_per_step']); print({k: c.get(k) for k in ('registered','points','observations','median_reproj_px','max_centre_err_rel_radius','lm_steps','cg_iters','stage_s')})"
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['graph_checksum']); c=d['cfg5']; print(c.get('error'), c.get('value'), c.get('s_per_reconstruction'))"
