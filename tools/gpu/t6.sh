set -o pipefail
# T-build A/B (SFM_BA_TBUILD 0: one wave per group, 4 per block; 1: index chain pipelined; 2:
# pipelined, one wave per block; 3: not pipelined, one wave per block) at cfg5's final model.
OUT=gpurun_out/t6; mkdir -p $OUT
for v in 0 1 2 3; do
  SFM_BA_TBUILD=$v timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-cfg3 --no-fp64 --no-local --no-cpu-baseline > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { tail -30 $OUT/bench_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_$v.json').read().splitlines()[-1]); c=d['cfg5']; e=c['ba_rooflines']['explicit_schur']; print($v, e['schur_build'], e['setup_backsub_ms'], c.get('s_per_reconstruction'), c.get('points'), c.get('reproj_median_px', c.get('median_reproj_px')), c.get('ba_phase_s'))"
done
