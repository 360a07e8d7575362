set -o pipefail
# Round 4: the key-in-the-accumulator Hamming kernel for both orders — parity tests, then the
# ordered-pair timing (new kernel, and SFM_HAM_BOTH=fused for the A/B), interleaved twice.
OUT=gpurun_out/r6f; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_golden.py tests/test_gpu_host.py tests/test_gpu_orb.py tests/test_gpu_fullsize.py -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -30
tail -2 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 200 python -u tests/perf/ordered_pairs_time.py > $OUT/op_key_$r.json 2>> $OUT/op.err && cat $OUT/op_key_$r.json &&
  SFM_HAM_BOTH=fused timeout -k 10 200 python -u tests/perf/ordered_pairs_time.py > $OUT/op_fused_$r.json 2>> $OUT/op.err && cat $OUT/op_fused_$r.json || exit 1
done
for k in 500 2048; do K=$k timeout -k 10 200 python -u tests/perf/hamming_time.py > $OUT/ham_$k.json 2>> $OUT/op.err && cat $OUT/ham_$k.json || exit 1; done
