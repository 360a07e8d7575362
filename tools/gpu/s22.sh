# Round 6: scan units with the two-chunk static-LDS loop restored inside the unit loop — K1 tests,
# cfg2 call A/B (pre-units build / units / SFM_L2FR_UNITS=0), one PMC pass.
set -o pipefail
O=gpurun_out/s22; mkdir -p $O
export TMPDIR=/tmp
PREV=$PWD/sfm-project_amd/lib/libsfmcore_prev.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_match.py tests/test_gpu_fullsize.py > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $O/pytest.log | head -30; exit 1; }
for r in 1 2 3; do
  SFMCORE_LIB=$PREV timeout -k 10 120 python tests/perf/k1_cfg2_time.py ratio | sed 's/^/prev /' >> $O/cfg2_ab.txt || exit 1
  timeout -k 10 120 python tests/perf/k1_cfg2_time.py ratio | sed 's/^/units /' >> $O/cfg2_ab.txt || exit 1
  SFM_L2FR_UNITS=0 timeout -k 10 120 python tests/perf/k1_cfg2_time.py ratio | sed 's/^/units0 /' >> $O/cfg2_ab.txt || exit 1
done
cut -c1-80 $O/cfg2_ab.txt
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-include-regex "l2fr_scan" -d $O/pmc -o run --output-format csv -- python3 tests/perf/k1_cfg2_time.py ratio > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
python3 tools/pmc_summary.py $O/pmc > $O/pmc.txt && cat $O/pmc.txt
