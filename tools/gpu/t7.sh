set -o pipefail
# T-build A/B (SFM_BA_TBUILD 0: direct loads, four waves per block; 3: direct, one wave per block;
# 4: records staged in LDS by whole pieces) at cfg5's final model, then the BA GPU tests under 4.
OUT=gpurun_out/t7; mkdir -p $OUT
for v in 0 4 3; do
  SFM_BA_TBUILD=$v timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-cfg3 --no-fp64 --no-local --no-cpu-baseline > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { tail -30 $OUT/bench_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_$v.json').read().splitlines()[-1]); c=d['cfg5']; e=c['ba_rooflines']['explicit_schur']; print($v, round(e['schur_build']['ms'],4), round(e['schur_build']['frac'],3), round(e['setup_backsub_ms'],4), c.get('s_per_reconstruction'), c.get('points'), repr(c.get('mean_reproj_px')), c.get('ba_phase_s'))"
done
SFM_BA_TBUILD=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_ba_sharded.py tests/test_gpu_ba_lm.py tests/test_gpu_ba.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; exit $rc
