set -o pipefail
# Round 5: non-temporal u stores in the CG point pass (default) vs plain (BA_U_NT=0), interleaved:
# the BA step at the cfg5 final-model size and the cfg5 line's LM time.
OUT=gpurun_out/q5u; mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for v in base unt0; do
    L=""; [ $v != base ] && L=sfm-project_amd/lib/libsfmcore_$v.so
    SFMCORE_LIB=$L timeout -k 10 300 python -u tests/perf/ba_solve_bench.py 500 258000 4 > $OUT/$v.$i.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    grep '^{' $OUT/$v.$i.json | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$v', round(d['cg_iter_ms']*1000,2), round(d['chunked']['cg_iter_ms']*1000,2), round(d['setup_backsub_ms']*1000,1))"
    SFMCORE_LIB=$L timeout -k 10 400 python -u bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/cfg5_$v.$i.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/cfg5_$v.$i.json').read().splitlines()[-1]);c=d.get('cfg5',d);print('cfg5 $v', c.get('s_per_reconstruction'), c.get('ba_phase_s')['lm_s'], c['ba_rooflines']['cg_iteration'])"
  done
done
