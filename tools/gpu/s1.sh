# Round 6, K1 scan study: parity of the scan variants (L2 match tests), interleaved scan-only
# timing of variants + ablations, the cfg2 call, and one PMC pass per variant.
set -o pipefail
O=gpurun_out/s1; mkdir -p $O
LIB=$PWD/sfm-project_amd/lib
lib() { [ $1 = base ] && echo $LIB/libsfmcore.so || echo $LIB/libsfmcore_$1.so; }
for v in m16 c512 m16c512; do
  SFMCORE_LIB=$(lib $v) timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    -m gpu tests/test_gpu_match.py -k l2 > $O/pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -30 $O/pytest_$v.log; exit 1; }
  tail -1 $O/pytest_$v.log
done
for r in 1 2 3; do
  for v in base m16 c512 m16c512 noepi bare m16noepi m16bare nostage nolds; do
    SFMCORE_LIB=$(lib $v) timeout -k 10 120 python tests/perf/l2fr_scan_time.py >> $O/scan_time.txt 2>&1 || { echo "scan $v failed"; tail $O/scan_time.txt; exit 1; }
  done
done
cat $O/scan_time.txt
for v in base m16 c512 m16c512; do
  SFMCORE_LIB=$(lib $v) timeout -k 10 120 python tests/perf/k1_cfg2_time.py ratio | sed "s/^/$v /" >> $O/cfg2.txt || exit 1
done
cat $O/cfg2.txt
export TMPDIR=/tmp
for v in base m16 c512 noepi bare m16bare; do
  SFMCORE_LIB=$(lib $v) timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
    SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA \
    --kernel-include-regex l2fr_scan -d $O/pmc_$v -o run --output-format csv -- python3 tests/perf/l2fr_scan_time.py > $O/pmc_$v.log 2>&1 || { echo "pmc $v failed"; tail $O/pmc_$v.log; exit 1; }
  echo "== $v" >> $O/pmc.txt; python3 tools/pmc_summary.py $O/pmc_$v >> $O/pmc.txt
done
cat $O/pmc.txt
