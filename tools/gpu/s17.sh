# Round 6: single-block CG vector kernel (bas_pcg_vec1) A/B on cfg5; chunk-mode camera waves per
# camera (SFM_BA_CKW) on the random / local K3 problems and on cfg5's final model (ba_rooflines).
set -o pipefail
O=gpurun_out/s17; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_ba_lm.py tests/test_gpu_ba_sharded.py tests/test_gpu_ba.py tests/test_gpu_incremental.py > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $O/pytest.log | head -30; exit 1; }
for w in 1 2 8; do for v in random sorted; do SFM_BA_CKW=$w timeout -k 10 120 python tests/perf/ba_jtj_local.py 500 $v >> $O/jtj_local.jsonl || exit 1; done; done
python3 -c "
import json
for l in open('$O/jtj_local.jsonl'):
    d=json.loads(l); print(d['order'], 'ckw', d['ckw'], 'plain', round(d['plain_ms'],4), 'chunked', round(d['chunked_ms'],4))"
for r in 1 2; do
  for v in "base" "SFM_BA_VEC1=0" "SFM_BA_CKW=1" "SFM_BA_CKW=2"; do
    n=$(echo $v | tr ' =' '__')
    env $([ "$v" = base ] || echo $v) timeout -k 10 600 python bench.py --config cfg5 --steps 2 --warmup 1 > $O/cfg5_$n.$r.json 2> $O/cfg5_$n.$r.err || { tail -20 $O/cfg5_$n.$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/cfg5_$n.$r.json').read().splitlines()[-1]); c=d['cfg5']; b=c['ba_rooflines']; print('$n', round(c['s_per_reconstruction'],4), c['ba_phase_s']['lm_s'], c['ba_phase_s']['s'], c['points'], c['median_reproj_px'], c['lm_steps'], c['cg_iters'], 'k3', round(b['k3']['ms'],4), 'ck', round(b['chunked']['k3']['ms'],4), round(b['chunked']['k3']['frac'],3), 'cgit', round(b['explicit_schur']['cg_iteration']['ms'],4))"
  done
done
