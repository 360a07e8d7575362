# Round 6: scan units of UNIT pairs (2 default; variants 3, 4) — K1 tests, cfg2 call A/B against
# the pre-units build, one PMC pass per form.
set -o pipefail
O=gpurun_out/s23; mkdir -p $O
export TMPDIR=/tmp
PREV=$PWD/sfm-project_amd/lib/libsfmcore_prev.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_match.py tests/test_gpu_fullsize.py > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $O/pytest.log | head -30; exit 1; }
U3=$PWD/sfm-project_amd/lib/libsfmcore_unit3.so
U4=$PWD/sfm-project_amd/lib/libsfmcore_unit4.so
for r in 1 2 3; do
  SFMCORE_LIB=$PREV timeout -k 10 120 python tests/perf/k1_cfg2_time.py ratio | sed 's/^/prev /' >> $O/cfg2_ab.txt || exit 1
  timeout -k 10 120 python tests/perf/k1_cfg2_time.py ratio | sed 's/^/unit2 /' >> $O/cfg2_ab.txt || exit 1
  SFMCORE_LIB=$U3 timeout -k 10 120 python tests/perf/k1_cfg2_time.py ratio | sed 's/^/unit3 /' >> $O/cfg2_ab.txt || exit 1
  SFMCORE_LIB=$U4 timeout -k 10 120 python tests/perf/k1_cfg2_time.py ratio | sed 's/^/unit4 /' >> $O/cfg2_ab.txt || exit 1
done
cut -c1-90 $O/cfg2_ab.txt
for v in unit2 unit3 unit4; do
  L=""; [ $v = unit3 ] && L="SFMCORE_LIB=$U3"; [ $v = unit4 ] && L="SFMCORE_LIB=$U4"
  env $L timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-include-regex "l2fr_scan" -d $O/pmc_$v -o run --output-format csv -- python3 tests/perf/k1_cfg2_time.py ratio > $O/pmc_$v.log 2>&1 || { tail $O/pmc_$v.log; exit 1; }
  python3 tools/pmc_summary.py $O/pmc_$v > $O/pmc_$v.txt && echo "== $v" && grep -E "GRBM_GUI_ACTIVE|SQ_VALU_MFMA_BUSY" $O/pmc_$v.txt
done
