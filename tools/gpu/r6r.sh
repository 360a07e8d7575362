set -o pipefail
# Round 4: the ORB content cache of the per-pair drop-in: ORB GPU tests, then the reference's own
# pair loop over the drop-in with and without the cache.
OUT=gpurun_out/r6r; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_orb.py tests/test_gpu_host.py tests/test_gpu_golden.py -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_orb.log 2>&1
rc=$?
grep -E "FAILED|ERROR|^E  " $OUT/pytest_orb.log | head -20
tail -1 $OUT/pytest_orb.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tests/perf/reference_loop_time.py 12 > $OUT/loop.json 2> $OUT/loop.err || { tail -20 $OUT/loop.err; exit 1; }
cat $OUT/loop.json
