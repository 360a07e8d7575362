# Round 6: the ratio rule without cross check writes its output from the compaction (no final
# kernel) — K1 GPU tests, cfg2 call A/B against the previous build, kernel stats.
set -o pipefail
O=gpurun_out/s34; mkdir -p $O
export TMPDIR=/tmp
PREV=$PWD/sfm-project_amd/lib/libsfmcore_prev.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_match.py tests/test_gpu_fullsize.py > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $O/pytest.log | head -30; exit 1; }
for r in 1 2 3; do
  SFMCORE_LIB=$PREV timeout -k 10 120 python tests/perf/k1_cfg2_time.py ratio | sed 's/^/prev /' >> $O/cfg2_ab.txt || exit 1
  timeout -k 10 120 python tests/perf/k1_cfg2_time.py ratio | sed 's/^/new /' >> $O/cfg2_ab.txt || exit 1
done
cut -c1-90 $O/cfg2_ab.txt
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tests/perf/k1_cfg2_time.py ratio > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python3 - <<'PY'
import csv, re
for r in csv.DictReader(open('gpurun_out/s34/prof/run_kernel_stats.csv')):
    n = re.sub(r'\(.*', '', r['Name'].replace('(anonymous namespace)::', '').replace('void ', ''))
    if 'l2fr' in n: print(n, r['Calls'], round(float(r['AverageNs']) / 1e3, 1))
PY
