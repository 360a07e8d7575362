set -o pipefail
# Round 5: the BA step at the synthetic cfg5 size (500 x 100 k x 5) and at the
# cfg5 final-model size (500 x 258 k x 4), per CG iteration (unchunked and chunked) against
# 8 TB/s; then PMC of the CG point and camera passes.
OUT=gpurun_out/q5h; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tests/perf/ba_solve_bench.py > $OUT/ba_solve_100k.json 2> $OUT/ba_solve_100k.err || { tail -20 $OUT/ba_solve_100k.err; exit 1; }
timeout -k 10 300 python -u tests/perf/ba_solve_bench.py 500 258000 4 > $OUT/ba_solve_258k.json 2> $OUT/ba_solve_258k.err || { tail -20 $OUT/ba_solve_258k.err; exit 1; }
cat $OUT/ba_solve_100k.json $OUT/ba_solve_258k.json
timeout -k 10 900 bash tools/pmc_kernel.sh q5h_pcg "bas_pcg_point|bas_pcg_camera" "tests/perf/ba_solve_bench.py" > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
tail -60 $OUT/pmc.log
