set -o pipefail
# T-build A/B: SFM_BA_TBUILD 0 (all records staged by global_load_lds) vs 6 (W_b and V_d^-1 staged,
# W_a rows in registers one batch ahead: half the LDS), twice each; then the BA GPU tests under 6.
OUT=gpurun_out/t10; mkdir -p $OUT
i=0; for v in 0 6 0 6; do i=$((i+1))
  SFM_BA_TBUILD=$v timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-cfg3 --no-fp64 --no-local --no-cpu-baseline > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || { tail -30 $OUT/bench_${v}_$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_${v}_$i.json').read().splitlines()[-1]); c=d['cfg5']; e=c['ba_rooflines']['explicit_schur']; print('$v.$i', round(e['schur_build']['ms'],4), round(e['schur_build']['frac'],3), round(e['setup_backsub_ms'],4), c.get('s_per_reconstruction'), c.get('points'), repr(c.get('mean_reproj_px')), c.get('ba_phase_s'))"
done
SFM_BA_TBUILD=6 timeout -k 10 600 python -u -m pytest tests/test_gpu_ba_sharded.py tests/test_gpu_ba_lm.py tests/test_gpu_ba.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; exit $rc
