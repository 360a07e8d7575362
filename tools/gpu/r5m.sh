#!/bin/bash
# K2 (ransac.hip) compiled with the max-ilp scheduler strategy vs the default: interleaved
# tests/perf/ransac_variants.py (ordered schedule, cfg3, parity sample vs the oracle).
set -o pipefail
mkdir -p gpurun_out/r5m
export PYTHONUNBUFFERED=1 TMPDIR=/tmp MODES=0
for r in 1 2 3; do
  for v in base rilp; do
    L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
    echo -n "$v "; SFMCORE_LIB=$L timeout -k 10 200 python tests/perf/ransac_variants.py 2>&1 | grep "mode=" || exit 1
  done
done | tee gpurun_out/r5m/ab.txt
