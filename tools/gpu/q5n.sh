set -o pipefail
# Round 5: BA tests (incl. the sharding-invariance ones), then cfg5 kernel totals chunks 0 vs 8.
OUT=gpurun_out/q5n; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ba.py tests/test_gpu_ba_lm.py tests/test_gpu_ba_sharded.py tests/test_gpu_incremental.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for c in 0 8; do
  SFM_BA_CHUNKS=$c timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_c$c -o run --output-format csv -- python3 bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/c$c.log 2>&1 || { tail -20 $OUT/c$c.log; exit 1; }
  find $OUT/prof_c$c -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/stats_c$c.csv
  rm -rf $OUT/prof_c$c
done
python3 tools/kernel_stats_diff.py $OUT/stats_c0.csv $OUT/stats_c8.csv
grep -h '^{' $OUT/c0.log $OUT/c8.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); c=d.get('cfg5',d); print(c.get('s_per_reconstruction'), c.get('ba_phase_s'), c.get('median_reproj_px'))"
