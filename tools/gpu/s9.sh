# Round 6, K1 study 9: range info folded into the order kernel, recovery sub-batches 2; the
# 4-wave 32x32 scan (two blocks per CU) against the 8-wave one and the 16x16x64 4-wave form.
set -o pipefail
O=gpurun_out/s9; mkdir -p $O
LIB=$PWD/sfm-project_amd/lib
lib() { [ $1 = base ] && echo $LIB/libsfmcore.so || echo $LIB/libsfmcore_$1.so; }
for v in base w4; do
  SFMCORE_LIB=$(lib $v) timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    -m gpu tests/test_gpu_match.py tests/test_gpu_fullsize.py::test_cfg2_ratio_rule_every_pair > $O/pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
for r in 1 2 3; do
  for v in base w4 m16w4; do
    SFMCORE_LIB=$(lib $v) timeout -k 10 120 python tests/perf/k1_cfg2_time.py ratio | sed "s/^/$v /" >> $O/cfg2.txt || exit 1
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open('gpurun_out/s9/cfg2.txt'):
    v, j = l.split(' ', 1); d[v].append(round(json.loads(j)['ms_per_call'], 4))
for v, x in d.items(): print(v, x)
PY
for v in w4clk m16w4clk; do
  SFMCORE_LIB=$(lib $v) QB=512 WPS=1 timeout -k 10 120 python tests/perf/l2fr_clock.py >> $O/clock.jsonl || exit 1
done
python3 -c "
import json
for l in open('gpurun_out/s9/clock.jsonl'):
    d=json.loads(l); print(d['lib'], 'span', round(d['span_us'],1), 'clk', round(d['clock_ghz_median'],3), 'eff', round(d['kernel_mfma_eff'],3), 'block', {k: round(v,2) for k,v in d['block_us'].items()}, 'tail', round(d['cu_tail_us']['mean'],1))"
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tests/perf/k1_cfg2_time.py ratio > $O/prof.log 2>&1 || { echo "prof failed"; tail $O/prof.log; exit 1; }
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/s9/prof/run_kernel_stats.csv')):
    if 'l2fr' in r['Name']:
        print(f"  {r['Name'][:50]:50s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:9.1f} us")
PY
timeout -k 10 600 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_bench.py::test_bench_json_contract > $O/pytest_bench.log 2>&1; echo "bench contract rc=$?"; grep -E "PASS|FAIL|Error" $O/pytest_bench.log | tail -5
timeout -k 10 300 python -c "
import sys; sys.path.insert(0,'sfm-project_amd')
import sfmcore, json
ctx = sfmcore.context(0)
for t in (50, 200, 200):
    print(json.dumps(ctx.calib_mfma_i8(t)))
" > $O/calib.txt 2>&1; cat $O/calib.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_incremental.py::test_incremental_bench_cfg5_scene > $O/pytest_cfg5scene.log 2>&1; echo "cfg5 scene rc=$?"; grep -E "PASS|FAIL|Error|assert" $O/pytest_cfg5scene.log | tail -8
