set -o pipefail
# Round 5: explicit Schur — BA tests after the structure-build changes, then cfg5 (rooflines of the
# explicit path on the final model) with the explicit system on (auto) and off.
OUT=gpurun_out/q5x; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ba_lm.py tests/test_gpu_ba_sharded.py tests/test_gpu_incremental.py > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest.log | head -20; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for c in auto 0; do
  SFM_BA_SCHUR=$c timeout -k 10 400 python -u bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/cfg5_$c.json 2> $OUT/cfg5_$c.err || { tail -30 $OUT/cfg5_$c.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/cfg5_$c.json').read().splitlines()[-1]);c=d.get('cfg5',d);print('schur=$c', c.get('s_per_reconstruction'), c.get('ba_phase_s'), c.get('median_reproj_px')); print(json.dumps(c.get('ba_rooflines',{}).get('explicit_schur')))"
done
