# Round 6: LM step host overhead (tests/perf/ba_lm_host.py) with the problem bound to the context
# for the whole loop (BAProblem.bind) vs per call (SFM_BA_BIND=0); BA GPU tests on the new loop;
# cfg5 interleaved A/B; K3 graph-timed in the bench's BA rooflines.
set -o pipefail
O=gpurun_out/s13; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_ba_lm.py tests/test_gpu_ba_sharded.py tests/test_gpu_ba.py tests/test_gpu_incremental.py > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 1 0; do
  SFM_BA_BIND=$v timeout -k 10 300 python tests/perf/ba_lm_host.py 24 100 250 500 > $O/lm_host_bind$v.jsonl 2> $O/lm_host_bind$v.err || { tail -20 $O/lm_host_bind$v.err; exit 1; }
done
cat $O/lm_host_bind1.jsonl $O/lm_host_bind0.jsonl
for r in 1 2; do
  for v in 0 1; do
    SFM_BA_BIND=$v timeout -k 10 600 python bench.py --config cfg5 --steps 2 --warmup 1 > $O/cfg5_bind$v.$r.json 2> $O/cfg5_bind$v.$r.err || { tail -20 $O/cfg5_bind$v.$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/cfg5_bind$v.$r.json').read().splitlines()[-1]); c=d['cfg5']; print('bind=$v', round(c['s_per_reconstruction'],4), c['ba_phase_s'], c['points'], c['median_reproj_px'], c['lm_steps'], c['cg_iters'])"
  done
done
python3 -c "import json; d=json.loads(open('$O/cfg5_bind1.2.json').read().splitlines()[-1]); print(json.dumps(d['cfg5'].get('ba_rooflines'), indent=1))"
