# Round 6: forward scan by units of two pairs sharing the query image (build_units; the query
# fragments loaded once, the second pair's first chunk staged under the first's last, single-pair
# units dispatched last).  K1 GPU tests (bit-exact vs oracle / other paths), then cfg2 call time
# interleaved: pre-units build / units / SFM_L2FR_UNITS=0, kernel stats and one PMC pass.
set -o pipefail
O=gpurun_out/s21; mkdir -p $O
export TMPDIR=/tmp
PREV=$PWD/sfm-project_amd/lib/libsfmcore_prev.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_match.py tests/test_gpu_fullsize.py tests/test_gpu_ba_sharded.py > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $O/pytest.log | head -30; exit 1; }
for r in 1 2 3; do
  SFMCORE_LIB=$PREV timeout -k 10 120 python tests/perf/k1_cfg2_time.py ratio | sed 's/^/prev /' >> $O/cfg2_ab.txt || exit 1
  timeout -k 10 120 python tests/perf/k1_cfg2_time.py ratio | sed 's/^/units /' >> $O/cfg2_ab.txt || exit 1
  SFM_L2FR_UNITS=0 timeout -k 10 120 python tests/perf/k1_cfg2_time.py ratio | sed 's/^/units0 /' >> $O/cfg2_ab.txt || exit 1
done
cat $O/cfg2_ab.txt
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tests/perf/k1_cfg2_time.py ratio > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-include-regex "l2fr_scan" -d $O/pmc -o run --output-format csv -- python3 tests/perf/k1_cfg2_time.py ratio > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
python3 tools/pmc_summary.py $O/pmc > $O/pmc.txt && cat $O/pmc.txt
python3 - <<'PY'
import csv, re
for r in csv.DictReader(open('gpurun_out/s21/prof/run_kernel_stats.csv')):
    n = re.sub(r'\(.*', '', r['Name'].replace('(anonymous namespace)::', '').replace('void ', ''))
    if 'l2fr' in n: print(n, r['Calls'], round(float(r['AverageNs']) / 1e3, 1))
PY
