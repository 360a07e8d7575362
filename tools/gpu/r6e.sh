set -o pipefail
# Round 4: incremental / BA-sharded / bench tests after the device-side reprojection filter; the
# cfg5 line; rocprofv3 kernel stats of the ordered-pair timing (kernel vs finalize split).
OUT=gpurun_out/r6e; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_incremental.py tests/test_gpu_ba_sharded.py tests/test_gpu_bench.py -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -30
tail -2 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --config cfg5 --steps 3 --warmup 1 > $OUT/cfg5.json 2> $OUT/cfg5.err || { tail -30 $OUT/cfg5.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/cfg5.json').read().splitlines()[-1]); c=d['cfg5']; print(d['value'], d['ms_per_step']); print({k: c.get(k) for k in ('registered','points','observations','median_reproj_px','max_centre_err_rel_radius','lm_steps','cg_iters','stage_s')}); print([(b['n_obs'], b['lm_steps'], b['cg_iters'], round(b['s'],3), round(b['lm_s'],3)) for b in c['bundle_adjustments']])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_op -o run --output-format csv -- python3 tests/perf/ordered_pairs_time.py > $OUT/ordered_pairs.json 2> $OUT/ordered_pairs.err || { tail -20 $OUT/ordered_pairs.err; exit 1; }
cat $OUT/ordered_pairs.json
timeout -k 10 400 python -u bench.py --gpus 4 --dist-backend gloo --device 0 --steps 1 --warmup 1 --no-fp64 > $OUT/bench_n4_gloo.json 2> $OUT/bench_n4_gloo.err || { tail -20 $OUT/bench_n4_gloo.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_n4_gloo.json').read().splitlines()[-1]); print(d['n_gpus'], d['graph_checksum'], d['verified_matches_per_step'], d['distributed']['launcher'], [r['pairs'] for r in d['distributed']['per_rank']])"
