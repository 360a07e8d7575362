set -o pipefail
# Round 4: BA point-pass V_d^-1 loaded up front in the CG point pass (vipf, -DBA_VI_PREFETCH, since removed) vs base: the CG iteration at cfg5 scale
# (tests/perf/ba_solve_bench.py, 500 x 100 k x 5) and the cfg5 reconstruction, interleaved.
OUT=gpurun_out/r6w; mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for v in base vipf; do
    L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
    SFMCORE_LIB=$L timeout -k 10 200 python3 tests/perf/ba_solve_bench.py > $OUT/solve_${v}_$r.json 2> $OUT/solve_${v}_$r.err || { tail -20 $OUT/solve_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/solve_${v}_$r.json').read().splitlines()[-1]); print('$v', $r, 'cg_iter_us %.1f' % (d['cg_iter_ms']*1e3), 'frac %.3f' % d['roofline']['frac'], 'lm_step_ms %.3f' % d['lm_step_ms'], 'it6', d['cg_iters_to_1e-6'])"
    SFMCORE_LIB=$L timeout -k 10 300 python3 bench.py --config cfg5 --steps 3 --warmup 1 > $OUT/cfg5_${v}_$r.json 2> $OUT/cfg5_${v}_$r.err || { tail -20 $OUT/cfg5_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/cfg5_${v}_$r.json').read().splitlines()[-1]); c=d['cfg5']; print('$v', $r, 'cfg5 s %.4f' % c['s_per_reconstruction'], c['ba_phase_s'], 'pts', c['points'], 'med %.6f' % c['median_reproj_px'], 'cg', c['cg_iters'], 'lm', c['lm_steps'])"
  done
done
