# Round 6, K1 study 8: SWAR-sorted recovery (sub-batches 4 vs 2), query-image block order,
# in-kernel stamps with the MFMA-block priority; parity, cfg2 timing, kernel stats.
set -o pipefail
O=gpurun_out/s8; mkdir -p $O
LIB=$PWD/sfm-project_amd/lib
lib() { [ $1 = base ] && echo $LIB/libsfmcore.so || echo $LIB/libsfmcore_$1.so; }
for v in base qord recsb2; do
  SFMCORE_LIB=$(lib $v) timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    -m gpu tests/test_gpu_match.py -k l2 tests/test_gpu_fullsize.py::test_cfg2_ratio_rule_every_pair > $O/pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
for r in 1 2 3; do
  for v in base qord recsb2 m16w4 m16w4qord; do
    SFMCORE_LIB=$(lib $v) timeout -k 10 120 python tests/perf/k1_cfg2_time.py ratio | sed "s/^/$v /" >> $O/cfg2.txt || exit 1
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open('gpurun_out/s8/cfg2.txt'):
    v, j = l.split(' ', 1); d[v].append(round(json.loads(j)['ms_per_call'], 4))
for v, x in d.items(): print(v, x)
PY
for v in clk qordclk; do
  SFMCORE_LIB=$(lib $v) timeout -k 10 120 python tests/perf/l2fr_clock.py >> $O/clock.jsonl || exit 1
done
cat $O/clock.jsonl
export TMPDIR=/tmp
for v in base recsb2 qord; do
  SFMCORE_LIB=$(lib $v) timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 tests/perf/k1_cfg2_time.py ratio > $O/prof_$v.log 2>&1 || { echo "prof failed"; tail $O/prof_$v.log; exit 1; }
  python3 - $v <<'PY'
import csv, sys
v = sys.argv[1]
for r in csv.DictReader(open(f'gpurun_out/s8/prof_{v}/run_kernel_stats.csv')):
    if 'l2fr' in r['Name']:
        print(f"  {v} {r['Name'][:50]:50s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:9.1f} us")
PY
done
