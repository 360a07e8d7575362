# Round 6, K1 study 3: parity of the MFMA recovery (+ the scan variants) on the L2 match tests,
# interleaved cfg2 call timing (recovery VALU vs MFMA; scan 32x32 / 16x16x64; 8- / 4-wave blocks),
# and in-kernel stamps of the 4-wave forms.
set -o pipefail
O=gpurun_out/s3; mkdir -p $O
LIB=$PWD/sfm-project_amd/lib
lib() { [ $1 = base ] && echo $LIB/libsfmcore.so || echo $LIB/libsfmcore_$1.so; }
for v in base m16 w4 m16w4; do
  SFMCORE_LIB=$(lib $v) timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    -m gpu tests/test_gpu_match.py -k l2 > $O/pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
for r in 1 2 3; do
  for v in base rvalu m16 w4 m16w4; do
    SFMCORE_LIB=$(lib $v) timeout -k 10 120 python tests/perf/k1_cfg2_time.py ratio | sed "s/^/$v /" >> $O/cfg2.txt || exit 1
  done
done
cat $O/cfg2.txt
for v in w4clk m16w4clk; do
  SFMCORE_LIB=$(lib $v) QB=512 WPS=1 timeout -k 10 120 python tests/perf/l2fr_clock.py >> $O/clock.jsonl || exit 1
done
cat $O/clock.jsonl
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tests/perf/k1_cfg2_time.py ratio > $O/prof.log 2>&1 || { echo "prof failed"; tail $O/prof.log; exit 1; }
SFMCORE_LIB=$(lib m16w4) timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/prof_m16w4 -o run --output-format csv -- python3 tests/perf/k1_cfg2_time.py ratio > $O/prof_m16w4.log 2>&1 || { echo "prof failed"; tail $O/prof_m16w4.log; exit 1; }
