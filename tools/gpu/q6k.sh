set -o pipefail
# Round 5: upload paths of the cfg5 descriptor set.
OUT=gpurun_out/q6k; mkdir -p $OUT
timeout -k 10 200 python -u tests/perf/upload_time.py > $OUT/upload.log 2>&1 || { tail -20 $OUT/upload.log; exit 1; }
cat $OUT/upload.log
