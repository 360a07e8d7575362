#!/bin/bash
# ORB select-kernel phase ablations (timing-only builds) + the default ORB bench (64 images 1080p).
set -o pipefail
mkdir -p gpurun_out/r4b
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python tests/perf/orb_bench.py > gpurun_out/r4b_orb_bench.json 2> gpurun_out/r4b_orb_bench.err || exit 1
for r in 1 2; do
  for v in base orb_HARRIS orb_DESC orb_SELECT; do
    L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
    SFMCORE_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4b/${v}_$r -o run -- python3 tests/perf/orb_bench.py 32 > gpurun_out/r4b/${v}_$r.log 2>&1 || exit 1
    python3 tools/orb_kstats.py gpurun_out/r4b/${v}_$r $v
  done
done
