set -o pipefail
# Round 5: cfg5 BA phases with the chunk table off / on, interleaved (entry wait, problem set-up).
OUT=gpurun_out/q5p; mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for c in 0 8; do
    SFM_BA_CHUNKS=$c timeout -k 10 400 python -u bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/c$c.$i.json 2> $OUT/c$c.$i.err || { tail -30 $OUT/c$c.$i.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/c$c.$i.json').read().splitlines()[-1]);c=d.get('cfg5',d);print('chunks=$c', c.get('s_per_reconstruction'), c.get('ba_phase_s'), c.get('median_reproj_px'))"
  done
done
