#!/bin/bash
# ORB tile kernel phase ablations after the blur/NMS rework (timing-only builds), rocprofv3 stats,
# 32 images 1080p, two interleaved rounds.
set -o pipefail
mkdir -p gpurun_out/r3w
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for r in 1 2; do
  for v in base orb_FILL orb_COMPASS orb_FAST; do
    L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
    SFMCORE_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3w/${v}_$r -o run -- python3 tests/perf/orb_bench.py 32 > gpurun_out/r3w/${v}_$r.log 2>&1 || exit 1
    python3 tools/orb_kstats.py gpurun_out/r3w/${v}_$r $v
  done
done
