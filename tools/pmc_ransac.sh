#!/bin/bash
# PMC passes over tests/perf/ransac_variants.py for the K2 hypothesis kernel (one counter group per pass).
set -o pipefail
TAG=${1:-pmc_ransac}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INST_CYCLES_SMEM SQ_ACTIVE_INST_SCA SQ_THREAD_CYCLES_VALU SQ_IFETCH GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "ransac_hyp|ransac_score|ransac_fit" -d $OUT/p$i -o run --output-format csv -- python3 tests/perf/ransac_variants.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
find $OUT -name "*counter_collection.csv" | head
