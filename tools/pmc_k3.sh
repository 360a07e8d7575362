#!/bin/bash
# K3 at cfg5 (tests/perf/ba_bench.py): kernel-trace stats and PMC passes (one counter group per
# pass, kernel trace only) for the library in $SFMCORE_LIB (default build if unset).
# Usage: tools/pmc_k3.sh TAG KERNEL_REGEX
set -o pipefail
TAG=${1:-pmc_k3}
KRE=${2:-ba_}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || { echo "rocprofv3 -L failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 tests/perf/ba_bench.py > $OUT/stats.log 2>&1 || { echo "stats pass failed"; tail -5 $OUT/stats.log; exit 1; }
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  keep=""
  for c in $set; do grep -qw "$c" $OUT/counters.txt && keep="$keep $c"; done
  echo "pass $i:$keep"
  timeout -k 10 300 rocprofv3 --pmc $keep --kernel-include-regex "$KRE" -d $OUT/p$i -o run --output-format csv -- python3 tests/perf/ba_bench.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
