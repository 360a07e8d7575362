set -o pipefail
# Round 5: BA tests, then the BA step timings at the cfg5 final-model size (CG camera-pass MLP).
OUT=gpurun_out/q5q; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ba.py tests/test_gpu_ba_lm.py tests/test_gpu_ba_sharded.py tests/test_gpu_incremental.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u tests/perf/ba_solve_bench.py 500 258000 4 > $OUT/ba_solve_258k.json 2> $OUT/ba_solve_258k.err || { tail -20 $OUT/ba_solve_258k.err; exit 1; }
grep '^{' $OUT/ba_solve_258k.json | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('cg_iter_ms', d['cg_iter_ms'], 'frac', d['roofline']['frac'], 'chunked', d['chunked'])"
