#!/bin/bash
# L2 / scalar-cache counters of ransac_score_kernel (mode 0, cfg3 ransac_variants.py): where its
# memory fetches come from.  One counter group per pass.
set -o pipefail
OUT=gpurun_out/${1:-pmc_ransac_l2}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for set in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" \
           "TCC_REQ_sum TCC_READ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE" \
           "SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_TC_DATA_READ_REQ"; do
  i=$((i+1))
  MODES=0 timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "ransac_score" -d $OUT/p$i -o run --output-format csv -- python3 tests/perf/ransac_variants.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
find $OUT -name "*counter_collection.csv" | head
