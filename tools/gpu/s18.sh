# Round 6: look-ahead CG poll (SFM_BA_POLL_AHEAD) and the speculative next linearisation
# (SFM_BA_SPEC) on top of the registered-camera compaction and the poll hint; chunk mode's camera
# waves now G = 1 at 500 cameras.  BA / incremental GPU tests, then cfg5 interleaved A/B against
# each knob off and against all of round 6's LM changes off.
set -o pipefail
O=gpurun_out/s18; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_ba_lm.py tests/test_gpu_ba_sharded.py tests/test_gpu_ba.py tests/test_gpu_incremental.py > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $O/pytest.log | head -30; exit 1; }
for r in 1 2 3; do
  for v in "base" "SFM_BA_SPEC=0" "SFM_BA_POLL_AHEAD=0" "SFM_BA_SPEC=0 SFM_BA_POLL_AHEAD=0 SFM_BA_POLL_HINT=0 SFM_BA_COMPACT=0"; do
    n=$(echo $v | tr ' =' '__')
    env $([ "$v" = base ] || echo $v) timeout -k 10 600 python bench.py --config cfg5 --steps 2 --warmup 1 > $O/cfg5_$n.$r.json 2> $O/cfg5_$n.$r.err || { tail -20 $O/cfg5_$n.$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/cfg5_$n.$r.json').read().splitlines()[-1]); c=d['cfg5']; b=c['ba_rooflines']; print('$n'[:60], round(c['s_per_reconstruction'],4), c['ba_phase_s']['lm_s'], c['ba_phase_s']['s'], c['points'], c['median_reproj_px'], c['lm_steps'], c['cg_iters'], 'ck', round(b['chunked']['k3']['ms'],4), round(b['chunked']['k3']['frac'],3))"
  done
done
