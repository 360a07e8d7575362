# Round 6: (a) the fused one-launch explicit CG iteration (bas_schur_iter) — BA / incremental GPU
# tests, LM host study and cfg5 A/B against SFM_BA_FUSE=0; (b) K3 chunk mode on a cfg5-like local
# visibility problem: plain vs chunked, camera waves per camera, observation-only / camera-only
# ablation builds.
set -o pipefail
O=gpurun_out/s15; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_ba_lm.py tests/test_gpu_ba_sharded.py tests/test_gpu_ba.py tests/test_gpu_incremental.py > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in sorted random; do timeout -k 10 120 python tests/perf/ba_jtj_local.py 500 $v >> $O/jtj_local.jsonl || exit 1; done
for w in 1 2 4; do SFM_BA_CKW=$w timeout -k 10 120 python tests/perf/ba_jtj_local.py 500 sorted >> $O/jtj_local.jsonl || exit 1; done
for v in obsonly camonly; do SFMCORE_LIB=$PWD/sfm-project_amd/lib/libsfmcore_$v.so timeout -k 10 120 python tests/perf/ba_jtj_local.py 500 sorted >> $O/jtj_local.jsonl || exit 1; done
cat $O/jtj_local.jsonl
for v in 1 0; do
  SFM_BA_FUSE=$v timeout -k 10 300 python tests/perf/ba_lm_host.py 100 250 500 > $O/lm_host_fuse$v.jsonl 2> $O/lm_host_fuse$v.err || { tail -20 $O/lm_host_fuse$v.err; exit 1; }
done
python3 - <<'PY'
import json
for v in (1, 0):
    for l in open(f'gpurun_out/s15/lm_host_fuse{v}.jsonl'):
        d = json.loads(l)
        print('fuse', v, d['n_cam'], 'solve gpu us', round(d['solve']['gpu_us'], 1), 'lm us/step', round(d['ba']['lm_us_per_step']), d['ba']['cg_iters'])
PY
for r in 1 2; do
  for v in 0 1; do
    SFM_BA_FUSE=$v timeout -k 10 600 python bench.py --config cfg5 --steps 2 --warmup 1 > $O/cfg5_fuse$v.$r.json 2> $O/cfg5_fuse$v.$r.err || { tail -20 $O/cfg5_fuse$v.$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/cfg5_fuse$v.$r.json').read().splitlines()[-1]); c=d['cfg5']; print('fuse=$v', round(c['s_per_reconstruction'],4), c['ba_phase_s'], c['points'], c['median_reproj_px'], c['lm_steps'], c['cg_iters'], c['ba_rooflines']['explicit_schur']['cg_iteration']['ms'])"
  done
done
