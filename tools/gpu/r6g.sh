set -o pipefail
# Debug of ham_key_kernel: the Hamming parity tests with the query constant from the extra MFMA
# k-step (base) and from the VALU (variant vq).
OUT=gpurun_out/r6g; mkdir -p $OUT
for v in base vq; do
  L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
  SFMCORE_LIB=$L timeout -k 10 200 python -u -m pytest tests/test_gpu_match.py -k "hamming_ragged or hamming_reference or both_orders_hamming" -q -p no:cacheprovider --timeout 100 --timeout-method thread > $OUT/pytest_$v.log 2>&1
  echo "$v rc=$?: $(tail -1 $OUT/pytest_$v.log)"
  grep -E "^E " $OUT/pytest_$v.log | head -6
done
