# Round 6, K1 study 4: parity + timing of the latency-built MFMA recovery, and the MFMA-block
# priority variants of the scan (32x32 / 16x16x64, 8- / 4-wave blocks).
set -o pipefail
O=gpurun_out/s6; mkdir -p $O
LIB=$PWD/sfm-project_amd/lib
lib() { [ $1 = base ] && echo $LIB/libsfmcore.so || echo $LIB/libsfmcore_$1.so; }
for v in base mprio; do
  SFMCORE_LIB=$(lib $v) timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    -m gpu tests/test_gpu_match.py -k l2 > $O/pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
for r in 1 2 3; do
  for v in base mprio m16w4mprio; do
    SFMCORE_LIB=$(lib $v) timeout -k 10 120 python tests/perf/k1_cfg2_time.py ratio | sed "s/^/$v /" >> $O/cfg2.txt || exit 1
  done
done
cat $O/cfg2.txt
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tests/perf/k1_cfg2_time.py ratio > $O/prof.log 2>&1 || { echo "prof failed"; tail $O/prof.log; exit 1; }
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/s6/prof/run_kernel_stats.csv')):
    print(f"  {r['Name'][:60]:60s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:9.1f} us")
PY
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py -k cfg2 tests/test_gpu_bench.py::test_bench_cfg4_line_carries_cfg5_at_two_ranks tests/test_gpu_ba_sharded.py::test_ba_sharded_more_ranks_than_chunks tests/test_gpu_ransac.py::test_ransac_stats_identity > $O/pytest_new.log 2>&1; echo "new tests rc=$?"; tail -15 $O/pytest_new.log
