# Round 6, K1 study 7: the prefix-sorted MFMA recovery; base (32x32, MFMA-block priority) vs the
# 16x16x64 4-wave form: parity, cfg2 timing, kernel stats and one PMC pass each; the new tests.
set -o pipefail
O=gpurun_out/s7; mkdir -p $O
LIB=$PWD/sfm-project_amd/lib
lib() { [ $1 = base ] && echo $LIB/libsfmcore.so || echo $LIB/libsfmcore_$1.so; }
for v in base m16w4; do
  SFMCORE_LIB=$(lib $v) timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    -m gpu tests/test_gpu_match.py -k l2 > $O/pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
for r in 1 2 3; do
  for v in base m16w4; do
    SFMCORE_LIB=$(lib $v) timeout -k 10 120 python tests/perf/k1_cfg2_time.py ratio | sed "s/^/$v /" >> $O/cfg2.txt || exit 1
  done
done
cat $O/cfg2.txt
export TMPDIR=/tmp
for v in base m16w4; do
  SFMCORE_LIB=$(lib $v) timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 tests/perf/k1_cfg2_time.py ratio > $O/prof_$v.log 2>&1 || { echo "prof failed"; tail $O/prof_$v.log; exit 1; }
  SFMCORE_LIB=$(lib $v) timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
    SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA \
    --kernel-include-regex "l2fr_scan|l2fr_recover" -d $O/pmc_$v -o run --output-format csv -- python3 tests/perf/k1_cfg2_time.py ratio > $O/pmc_$v.log 2>&1 || { echo "pmc $v failed"; tail $O/pmc_$v.log; exit 1; }
  echo "== $v" >> $O/pmc.txt; python3 tools/pmc_summary.py $O/pmc_$v >> $O/pmc.txt
  python3 - $v <<'PY'
import csv, sys
v = sys.argv[1]
for r in csv.DictReader(open(f'gpurun_out/s7/prof_{v}/run_kernel_stats.csv')):
    print(f"  {v} {r['Name'][:60]:60s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:9.1f} us")
PY
done
cat $O/pmc.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_bench.py::test_bench_cfg4_line_carries_cfg5_at_two_ranks tests/test_gpu_ba_sharded.py::test_ba_sharded_more_ranks_than_chunks tests/test_gpu_ransac.py::test_ransac_stats_identity > $O/pytest_new.log 2>&1; echo "new tests rc=$?"; grep -E "PASS|FAIL|Error|error" $O/pytest_new.log | tail -20
for r in 1 2; do
  for v in base mumprio; do
    SFMCORE_LIB=$(lib $v) K1_ONLY_BENCH_RULE=1 timeout -k 10 120 python tests/perf/k1_time.py 2>&1 | grep "xc=" | sed "s/^/$v cfg3 /" >> $O/mu_ab.txt || exit 1
  done
done
cat $O/mu_ab.txt
for v in base mumprio m16w4; do
  SFMCORE_LIB=$(lib $v) timeout -k 10 300 python tests/perf/k1_mutual_ab.py >> $O/mutual_fr_cfg4.jsonl || exit 1
done
cat $O/mutual_fr_cfg4.jsonl
