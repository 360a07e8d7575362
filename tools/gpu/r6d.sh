set -o pipefail
# Round 4: incremental / BA / bench / host GPU tests after the LM function tolerance and the
# device-side CSR; the cfg5 line on its own; then rocprofv3 kernel stats of the default bench.
OUT=gpurun_out/r6d; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_incremental.py tests/test_gpu_ba_lm.py tests/test_gpu_ba_sharded.py tests/test_gpu_bench.py tests/test_gpu_host.py tests/test_gpu_recon.py -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -30
tail -2 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --config cfg5 --steps 2 --warmup 1 > $OUT/cfg5.json 2> $OUT/cfg5.err || { tail -30 $OUT/cfg5.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/cfg5.json').read().splitlines()[-1]); c=d['cfg5']; print(d['value'], d['ms_per_step']); print({k: c.get(k) for k in ('registered','points','observations','median_reproj_px','max_centre_err_rel_radius','lm_steps','cg_iters','stage_s')}); print([(b['n_obs'], b['lm_steps'], b['cg_iters'], round(b['s'],3), round(b['lm_s'],3)) for b in c['bundle_adjustments']])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['ms']); c=d['cfg5']; print(c.get('error'), c.get('value'), c.get('s_per_reconstruction'))"
find $OUT/prof -name "*kernel_stats.csv" | head -3
