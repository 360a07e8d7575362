set -o pipefail
# Round 5 (final driver): cfg5 at full size, N = 1 and the 2-rank job
# through the self-launcher's count-then-spawn path (gloo, both ranks on this GPU).
OUT=gpurun_out/q6o; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/n1.json 2> $OUT/n1.err || { tail -30 $OUT/n1.err; exit 1; }
timeout -k 10 900 python -u bench.py --config cfg5 --steps 1 --warmup 1 --gpus 2 --ranks-per-gpu 2 --dist-backend gloo --no-cpu-baseline > $OUT/n2.json 2> $OUT/n2.err || { tail -30 $OUT/n2.err; exit 1; }
python3 - <<'PY'
import json
a = json.loads(open("gpurun_out/q6o/n1.json").read().splitlines()[-1])
b = json.loads(open("gpurun_out/q6o/n2.json").read().splitlines()[-1])
a, b = a.get("cfg5", a), b.get("cfg5", b)
for k in ("registered", "points", "verified_matches", "median_reproj_px", "mean_reproj_px", "s_per_reconstruction", "ba_phase_s", "pcg_branches", "stage_s"):
    print(k, a.get(k), b.get(k))
PY
