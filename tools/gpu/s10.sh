# Round 6, K1 study 10: the persistent forward scan (next unit's first chunk + waves 0-3's query
# rows staged during the last chunk) and the one-record unit decode; parity, cfg2 timing, PMC.
set -o pipefail
O=gpurun_out/s10; mkdir -p $O
LIB=$PWD/sfm-project_amd/lib
lib() { [ $1 = base ] && echo $LIB/libsfmcore.so || echo $LIB/libsfmcore_$1.so; }
for v in persist base; do
  SFMCORE_LIB=$(lib $v) timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    -m gpu tests/test_gpu_match.py tests/test_gpu_fullsize.py::test_cfg2_ratio_rule_every_pair > $O/pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
for r in 1 2 3; do
  for v in base persist; do
    SFMCORE_LIB=$(lib $v) timeout -k 10 120 python tests/perf/k1_cfg2_time.py ratio | sed "s/^/$v /" >> $O/cfg2.txt || exit 1
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open('gpurun_out/s10/cfg2.txt'):
    v, j = l.split(' ', 1); d[v].append(round(json.loads(j)['ms_per_call'], 4))
for v, x in d.items(): print(v, x)
PY
export TMPDIR=/tmp
for v in base persist; do
  SFMCORE_LIB=$(lib $v) timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 tests/perf/k1_cfg2_time.py ratio > $O/prof_$v.log 2>&1 || { echo "prof failed"; tail $O/prof_$v.log; exit 1; }
  SFMCORE_LIB=$(lib $v) timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-include-regex "l2fr_scan" -d $O/pmc_$v -o run --output-format csv -- python3 tests/perf/k1_cfg2_time.py ratio > $O/pmc_$v.log 2>&1 || { echo "pmc failed"; tail $O/pmc_$v.log; exit 1; }
  echo "== $v" >> $O/pmc.txt; python3 tools/pmc_summary.py $O/pmc_$v >> $O/pmc.txt
  python3 - $v <<'PY'
import csv, sys
v = sys.argv[1]
for r in csv.DictReader(open(f'gpurun_out/s10/prof_{v}/run_kernel_stats.csv')):
    if 'l2fr' in r['Name']:
        print(f"  {v} {r['Name'][:50]:50s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:9.1f} us")
PY
done
python3 - <<'PY'
import re
cur = None
for l in open('gpurun_out/s10/pmc.txt'):
    if l.startswith('=='): cur = l.strip()
    m = re.match(r'\s+(\w+)\s+([\d.]+)', l)
    if m: globals().setdefault('vals', {}).setdefault(cur, {})[m.group(1)] = float(m.group(2))
for k, d in vals.items():
    print(k, 'MFMA busy', round(d['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * d['GRBM_GUI_ACTIVE'] / 8), 4))
PY
