# Round 6: the reprojection errors from the LM's last speculative K3 — BA / incremental GPU tests
# and the cfg5 line twice.
set -o pipefail
O=gpurun_out/s27; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_ba_lm.py tests/test_gpu_ba_sharded.py tests/test_gpu_ba.py tests/test_gpu_incremental.py > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $O/pytest.log | head -30; exit 1; }
for r in 1 2; do
  timeout -k 10 600 python bench.py --config cfg5 --steps 2 --warmup 1 > $O/cfg5.$r.json 2> $O/cfg5.$r.err || { tail -20 $O/cfg5.$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/cfg5.$r.json').read().splitlines()[-1]); c=d['cfg5']; print(round(c['s_per_reconstruction'],4), c['ba_phase_s'], c['points'], c['median_reproj_px'], c['lm_steps'], c['cg_iters'])"
done
