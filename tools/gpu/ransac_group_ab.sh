#!/bin/bash
# A/B of the ordered RANSAC schedule's pair-group size (SFM_RANSAC_GROUP, ransac.hip
# xcd_pair_block): K2 ms of the cfg4 bench step and the cfg3 launch, interleaved.
# Usage: tools/gpu/ransac_group_ab.sh TAG "0 32 64 128"
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
for rep in 1 2; do
  for g in $2; do
    SFM_RANSAC_GROUP=$g timeout -k 10 240 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cfg3 > $OUT/cfg4_g${g}_r$rep.json 2> $OUT/cfg4_g${g}_r$rep.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('cfg4 group', sys.argv[2], 'ransac_ms %.3f' % d['stages']['ransac_ms'], 'step_ms %.2f' % d['ms_per_step'])" $OUT/cfg4_g${g}_r$rep.json $g | tee -a $OUT/summary.txt
    SFM_RANSAC_GROUP=$g MODES=0 timeout -k 10 200 python3 tests/perf/ransac_variants.py 2>&1 | sed "s/^/cfg3 group $g /" | tee -a $OUT/summary.txt || exit 1
  done
done
