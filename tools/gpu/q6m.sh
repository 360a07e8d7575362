set -o pipefail
# Round 5: speculative next linearisation in the LM loop: incremental tests, BA set-up cost, cfg5 leg.
OUT=gpurun_out/q6m; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_incremental.py tests/test_gpu_ba_lm.py tests/test_gpu_ba_sharded.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 500 python -u bench.py --config cfg5 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/cfg5.json 2> $OUT/cfg5.err || { tail -20 $OUT/cfg5.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/q6m/cfg5.json").read().strip().splitlines()[-1])
c = d.get("cfg5", d)
print(c.get("s_per_reconstruction"), c.get("walls_s_rank"), c.get("stage_s"), c.get("ba_phase_s"), c.get("registered"), c.get("points"), c.get("median_reproj_px"))
PY
