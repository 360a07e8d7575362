# Round 6, K1 scan study 2: in-kernel stamps of the forward scan (32x32 and 16x16x64 forms) at
# cfg2 (50 x 2048) and 25 x 4096, and interleaved timing of the static-priority variants.
set -o pipefail
O=gpurun_out/s2; mkdir -p $O
LIB=$PWD/sfm-project_amd/lib
lib() { [ $1 = base ] && echo $LIB/libsfmcore.so || echo $LIB/libsfmcore_$1.so; }
for v in clk m16clk; do
  SFMCORE_LIB=$(lib $v) timeout -k 10 120 python tests/perf/l2fr_clock.py >> $O/clock.jsonl || exit 1
  SFMCORE_LIB=$(lib $v) N_IMG=25 K=4096 timeout -k 10 120 python tests/perf/l2fr_clock.py >> $O/clock.jsonl || exit 1
done
cat $O/clock.jsonl
for r in 1 2 3; do
  for v in base m16 prio m16prio; do
    SFMCORE_LIB=$(lib $v) timeout -k 10 120 python tests/perf/l2fr_scan_time.py 2>&1 | grep scan-only >> $O/scan_time.txt || exit 1
    SFMCORE_LIB=$(lib $v) N_IMG=25 K=4096 timeout -k 10 120 python tests/perf/l2fr_scan_time.py 2>&1 | grep scan-only | sed 's/^/k4096 /' >> $O/scan_time.txt || exit 1
  done
done
cat $O/scan_time.txt
