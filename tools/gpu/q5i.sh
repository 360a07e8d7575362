set -o pipefail
# Round 5: chunk-mode BA after the halving wave sums and the folded chunk finish — BA tests
# (single, sharded bit-identity, incremental sharding invariance) then the BA step timings.
OUT=gpurun_out/q5i; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ba.py tests/test_gpu_ba_lm.py tests/test_gpu_ba_sharded.py tests/test_gpu_incremental.py tests/test_gpu_recon.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python -u tests/perf/ba_solve_bench.py > $OUT/ba_solve_100k.json 2> $OUT/ba_solve_100k.err || { tail -20 $OUT/ba_solve_100k.err; exit 1; }
timeout -k 10 300 python -u tests/perf/ba_solve_bench.py 500 258000 4 > $OUT/ba_solve_258k.json 2> $OUT/ba_solve_258k.err || { tail -20 $OUT/ba_solve_258k.err; exit 1; }
grep '^{' $OUT/ba_solve_100k.json $OUT/ba_solve_258k.json
