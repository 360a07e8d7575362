set -o pipefail
# Round 5 (VERDICT r4 items 3 + 4): cfg5 at full size, N = 1 with the round-4 sums
# (SFM_BA_CHUNKS=0) and the sharding-invariant chunk sums interleaved, then the 2-rank job through
# the self-launcher (gloo, both ranks on this GPU).
OUT=gpurun_out/q5l; mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for c in 0 8; do
    SFM_BA_CHUNKS=$c timeout -k 10 400 python -u bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/n1_c$c.$i.json 2> $OUT/n1_c$c.$i.err || { tail -30 $OUT/n1_c$c.$i.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/n1_c$c.$i.json').read().splitlines()[-1]);c=d.get('cfg5',d);print('chunks=$c', c.get('s_per_reconstruction'), c.get('ba_phase_s'), c.get('median_reproj_px'), c.get('points'))"
  done
done
timeout -k 10 900 python -u bench.py --config cfg5 --steps 1 --warmup 1 --gpus 2 --ranks-per-gpu 2 --dist-backend gloo --no-cpu-baseline > $OUT/n2.json 2> $OUT/n2.err || { tail -30 $OUT/n2.err; exit 1; }
python3 - <<'PY'
import json
a = json.loads(open("gpurun_out/q5l/n1_c8.2.json").read().splitlines()[-1])
b = json.loads(open("gpurun_out/q5l/n2.json").read().splitlines()[-1])
a, b = a.get("cfg5", a), b.get("cfg5", b)
for k in ("registered", "points", "verified_matches", "median_reproj_px", "mean_reproj_px", "s_per_reconstruction", "ba_phase_s", "pcg_branches", "stage_s"):
    print(k, a.get(k), b.get(k))
PY
