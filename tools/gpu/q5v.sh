set -o pipefail
# Round 5: explicit reduced camera system — BA tests (explicit solve vs oracle / dense / implicit,
# duplicate camera + long tracks, sharded world-1 identity; the sharding-invariance tests now run
# it through bundle_adjust), then the cfg5 line.
OUT=gpurun_out/q5v; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ba_lm.py tests/test_gpu_ba.py tests/test_gpu_ba_sharded.py tests/test_gpu_incremental.py tests/test_gpu_recon.py > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error|error" $OUT/pytest.log | head -20; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for c in 0 auto; do
  SFM_BA_SCHUR=$c timeout -k 10 400 python -u bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/cfg5_$c.json 2> $OUT/cfg5_$c.err || { tail -30 $OUT/cfg5_$c.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/cfg5_$c.json').read().splitlines()[-1]);c=d.get('cfg5',d);print('schur=$c', c.get('s_per_reconstruction'), c.get('ba_phase_s'), c.get('median_reproj_px'), c.get('points'), c.get('lm_steps'), c.get('cg_iters'))"
done
