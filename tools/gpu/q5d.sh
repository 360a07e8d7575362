set -o pipefail
# Round 5: cfg5 at full size (500 x 4096) as a 2-rank job through the
# self-launcher's count-then-spawn path (gloo, both ranks on this GPU), and the N = 1 line.
OUT=gpurun_out/q5d; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --config cfg5 --steps 1 --warmup 1 > $OUT/cfg5_n1.json 2> $OUT/cfg5_n1.err || { tail -30 $OUT/cfg5_n1.err; exit 1; }
timeout -k 10 900 python -u bench.py --config cfg5 --steps 1 --warmup 1 --gpus 2 --ranks-per-gpu 2 --dist-backend gloo > $OUT/cfg5_n2.json 2> $OUT/cfg5_n2.err || { tail -30 $OUT/cfg5_n2.err; exit 1; }
python3 - <<'PY'
import json
a = json.loads(open("gpurun_out/q5d/cfg5_n1.json").read().splitlines()[-1])["cfg5"]
b = json.loads(open("gpurun_out/q5d/cfg5_n2.json").read().splitlines()[-1])["cfg5"]
for k in ("registered", "points", "verified_matches", "median_reproj_px", "mean_reproj_px", "s_per_reconstruction", "ba_phase_s", "pcg_branches"):
    print(k, a.get(k), b.get(k))
PY
