# Round 6: launches folded in the LM step (the fix kernels as one, the model chunk tree inside
# bas_model, the SoA copy inside the point set-up, the CG init inside the Schur tree launch,
# bas_model, p's zeroing inside the camera set-up; same bits) — BA tests, cfg5 A/B vs 355c465.
set -o pipefail
O=gpurun_out/s24; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_ba_lm.py tests/test_gpu_ba_sharded.py tests/test_gpu_ba.py tests/test_gpu_incremental.py > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $O/pytest.log | head -30; exit 1; }
for r in 1 2 3; do
  for v in prev base; do
    L=""; [ $v = prev ] && L="SFMCORE_LIB=$PWD/sfm-project_amd/lib/libsfmcore_prev.so"
    env $L timeout -k 10 600 python bench.py --config cfg5 --steps 2 --warmup 1 > $O/cfg5_$v.$r.json 2> $O/cfg5_$v.$r.err || { tail -20 $O/cfg5_$v.$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/cfg5_$v.$r.json').read().splitlines()[-1]); c=d['cfg5']; b=c['ba_rooflines']; print('$v', round(c['s_per_reconstruction'],4), c['ba_phase_s']['lm_s'], c['ba_phase_s']['s'], c['points'], c['median_reproj_px'], c['lm_steps'], c['cg_iters'], 'cgit', round(b['explicit_schur']['cg_iteration']['ms'],4), 'impl_cgit', round(b['cg_iteration']['ms'],4))"
  done
done
