#!/bin/bash
# PMC passes (one counter group per pass, kernel trace only) over a perf script (default
# tests/perf/k1_time.py) for the kernels matching KRE.  Usage: tools/pmc_kernel.sh TAG KRE [SCRIPT]
# Counters missing from `rocprofv3 -L` on the box are dropped from their pass.
set -o pipefail
TAG=${1:-pmc_k1}
KRE=${2:-mfma_match}
CMD=${3:-tests/perf/k1_time.py}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || { echo "rocprofv3 -L failed"; exit 1; }
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_VALU_MFMA_I8 SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  keep=""
  for c in $set; do grep -qw "$c" $OUT/counters.txt && keep="$keep $c"; done
  echo "pass $i:$keep"
  timeout -k 10 300 rocprofv3 --pmc $keep --kernel-include-regex "$KRE" -d $OUT/p$i -o run --output-format csv -- python3 $CMD > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
