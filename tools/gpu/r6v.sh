set -o pipefail
# Round 4: both orders from one tile at k_max 4096 (Hamming key kernel), GPU test.
OUT=gpurun_out/r6v; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py -k "both_orders" -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|^E  " $OUT/pytest.log | head -20
tail -1 $OUT/pytest.log
exit $rc
