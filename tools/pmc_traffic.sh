#!/bin/bash
# HBM traffic of the benchmark's kernels from rocprofv3 PMC, one counter per pass
# (FETCH_SIZE and WRITE_SIZE cannot share a pass), then tools/traffic_summary.py.
# Usage: tools/pmc_traffic.sh TAG [cfg3|cfg4]  -> gpurun_out/TAG/traffic.json
set -o pipefail
TAG=${1:-traffic}
CFG=${2:-cfg4}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
# launches per step: one per step at the bench default --chunk (131072), for both configs
if [ $CFG = cfg3 ]; then NI=50; K=2048; PER=1; else NI=500; K=4096; PER=1; fi
STEPS=2
B="python3 bench.py --config $CFG --steps $STEPS --warmup 1 --no-cpu-baseline --no-cfg3 --no-cfg5 --no-fp64 --no-local"
RX="mfma_prep_kernel|mfma_mutual_kernel|mutual_finalize_kernel|ransac_prep_kernel|ransac_fit_kernel|ransac_order_kernel|ransac_score_kernel|ransac_final_kernel|graph_rows_kernel"
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex "$RX" -d $OUT/p$i -o run --output-format csv -- $B > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/traffic_summary.py $OUT $CFG $NI $K $PER $STEPS > $OUT/traffic.json && cat $OUT/traffic.json
