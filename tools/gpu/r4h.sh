#!/bin/bash
# ORB tile-kernel phase ablations after the round-3 rework (timing-only builds), 32 images.
set -o pipefail
mkdir -p gpurun_out/r4h
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for r in 1 2; do
  for v in base orb_FILL orb_HBLUR orb_VBLUR orb_COMPASS orb_FAST orb_STORES; do
    L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
    SFMCORE_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4h/${v}_$r -o run -- python3 tests/perf/orb_bench.py 32 > gpurun_out/r4h/${v}_$r.log 2>&1 || exit 1
    python3 tools/orb_kstats.py gpurun_out/r4h/${v}_$r $v
  done
done
