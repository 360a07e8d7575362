set -o pipefail
# Round 4: single-copy verify_pair; host-layer GPU tests.
OUT=gpurun_out/r6y; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_host.py tests/test_gpu_ransac.py tests/test_gpu_golden.py -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|^E  " $OUT/pytest.log | head -20
tail -1 $OUT/pytest.log
exit $rc
