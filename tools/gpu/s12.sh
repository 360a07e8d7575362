# Round 6: the one-workgroup explicit CG (bas_schur_cg1, n_cam <= 256): BA / incremental GPU tests
# (bit-identity with the per-iteration kernels of the sharded path is part of them), then cfg5
# interleaved A/B against SFM_BA_CG1=0.
set -o pipefail
O=gpurun_out/s12; mkdir -p $O
timeout -k 10 1200 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_ba_lm.py tests/test_gpu_ba_sharded.py tests/test_gpu_ba.py tests/test_gpu_incremental.py > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in 0 1; do
    SFM_BA_CG1=$v timeout -k 10 600 python bench.py --config cfg5 --steps 2 --warmup 1 > $O/cfg5_cg1_$v.$r.json 2> $O/cfg5_cg1_$v.$r.err || { tail -20 $O/cfg5_cg1_$v.$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/cfg5_cg1_$v.$r.json').read().splitlines()[-1]); c=d['cfg5']; print('cg1=$v', round(c['s_per_reconstruction'],4), c['ba_phase_s'], c['points'], c['median_reproj_px'], c['lm_steps'], c['cg_iters'])"
  done
done
