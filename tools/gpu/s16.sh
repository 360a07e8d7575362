# Round 6: LM phase cuts — registered cameras only (SFM_BA_COMPACT), the convergence poll at the
# previous solve's iteration count (SFM_BA_POLL_HINT), the camera setup's tail over a wave, chunk
# mode's empty camera waves skipped.  BA / incremental / C-ABI GPU tests, K3 local study, cfg5 A/B.
set -o pipefail
O=gpurun_out/s16; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_ba_lm.py tests/test_gpu_ba_sharded.py tests/test_gpu_ba.py tests/test_gpu_incremental.py > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $O/pytest.log | head -30; }
for v in sorted random; do timeout -k 10 120 python tests/perf/ba_jtj_local.py 500 $v >> $O/jtj_local.jsonl || exit 1; done
SFM_BA_CKW=1 timeout -k 10 120 python tests/perf/ba_jtj_local.py 500 sorted >> $O/jtj_local.jsonl || exit 1
cat $O/jtj_local.jsonl
for r in 1 2; do
  for v in "base" "SFM_BA_COMPACT=0" "SFM_BA_POLL_HINT=0" "SFM_BA_COMPACT=0 SFM_BA_POLL_HINT=0"; do
    n=$(echo $v | tr ' =' '__')
    env $([ "$v" = base ] || echo $v) timeout -k 10 600 python bench.py --config cfg5 --steps 2 --warmup 1 > $O/cfg5_$n.$r.json 2> $O/cfg5_$n.$r.err || { tail -20 $O/cfg5_$n.$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/cfg5_$n.$r.json').read().splitlines()[-1]); c=d['cfg5']; b=c['ba_rooflines']; print('$n', round(c['s_per_reconstruction'],4), c['ba_phase_s'], c['points'], c['median_reproj_px'], c['lm_steps'], c['cg_iters'], 'k3', round(b['k3']['ms'],4), 'ck', round(b['chunked']['k3']['ms'],4), round(b['chunked']['k3']['frac'],3))"
  done
done
exit $rc
