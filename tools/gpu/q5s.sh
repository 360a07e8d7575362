set -o pipefail
# Round 5: CG point pass lanes per point (SFM_BA_PG 8 default vs 4), interleaved, cfg5 final size.
OUT=gpurun_out/q5s; mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for v in pg4 pg2 pg1; do
    L=""; [ $v != base ] && L=sfm-project_amd/lib/libsfmcore_$v.so
    SFMCORE_LIB=$L timeout -k 10 300 python -u tests/perf/ba_solve_bench.py 500 258000 4 > $OUT/$v.$i.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    grep '^{' $OUT/$v.$i.json | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$v', round(d['cg_iter_ms']*1000,2), round(d['chunked']['cg_iter_ms']*1000,2), round(d['setup_backsub_ms']*1000,1), d['cg_iters_to_1e-6'])"
  done
done
