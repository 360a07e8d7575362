set -o pipefail
# Round 5: CG point-pass lanes per point 8 (base) vs 4, on the cfg5 line and on the arc scene's
# incremental run (long tracks), interleaved.
OUT=gpurun_out/q5t; mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for v in base pg4; do
    L=""; [ $v != base ] && L=sfm-project_amd/lib/libsfmcore_$v.so
    SFMCORE_LIB=$L timeout -k 10 400 python -u bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/cfg5_$v.$i.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/cfg5_$v.$i.json').read().splitlines()[-1]);c=d.get('cfg5',d);print('cfg5 $v', c.get('s_per_reconstruction'), c.get('ba_phase_s'), c.get('median_reproj_px'), c.get('points'))"
    SFMCORE_LIB=$L timeout -k 10 400 python -u tests/perf/incremental_ba_probe.py > $OUT/arc_$v.$i.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/arc_$v.$i.json').read().splitlines()[-1]);print('arc $v wall', round(d['wall'],3), 'ba_s', round(sum(b['s'] for b in d['ba']),3), 'cg', sum(b['cg_total'] for b in d['ba']))"
  done
done
