set -o pipefail
# Round 5: fewer host syncs in the BA set-up: incremental tests, BA set-up cost, cfg5 leg.
OUT=gpurun_out/q6e; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_incremental.py tests/test_gpu_ba_lm.py tests/test_gpu_ba_sharded.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python -u tests/perf/ba_problem_time.py > $OUT/problem.log 2>&1 || { tail -20 $OUT/problem.log; exit 1; }
grep -v "^$" $OUT/problem.log | head -45
timeout -k 10 500 python -u bench.py --config cfg5 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/cfg5.json 2> $OUT/cfg5.err || { tail -20 $OUT/cfg5.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/q6e/cfg5.json").read().strip().splitlines()[-1])
c = d.get("cfg5", d)
print(c.get("s_per_reconstruction"), c.get("walls_s_rank"), c.get("stage_s"), c.get("ba_phase_s"), c.get("registered"), c.get("points"), c.get("median_reproj_px"))
PY
