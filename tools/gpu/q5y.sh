set -o pipefail
# Round 5: waves per (chunk, slot) group in the explicit Schur build (SB_WAVES 4 default, 2, 8):
# the cfg5 line's final-model T build and LM time.
OUT=gpurun_out/q5y; mkdir -p $OUT
export TMPDIR=/tmp
for v in base sb1; do
  L=""; [ $v != base ] && L=sfm-project_amd/lib/libsfmcore_$v.so
  SFMCORE_LIB=$L timeout -k 10 400 python -u bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/cfg5_$v.json 2> $OUT/cfg5_$v.err || { tail -30 $OUT/cfg5_$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/cfg5_$v.json').read().splitlines()[-1]);c=d.get('cfg5',d);e=c['ba_rooflines']['explicit_schur'];print('$v', c.get('s_per_reconstruction'), c['ba_phase_s']['lm_s'], c['ba_phase_s']['problem_s'], round(e['schur_build']['ms'],4), round(e['schur_build']['frac'],3), round(e['cg_iteration']['ms'],4))"
done
