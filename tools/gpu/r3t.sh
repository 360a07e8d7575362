#!/bin/bash
# ORB tile kernel: per-phase timing ablations (timing-only builds, wrong results by construction),
# rocprofv3 kernel stats of tests/perf/orb_bench.py (32 images 1080p), two interleaved rounds.
set -o pipefail
mkdir -p gpurun_out/r3t
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for r in 1 2; do
  for v in base orb_FILL orb_HBLUR orb_VBLUR orb_NMS orb_FAST; do
    L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
    SFMCORE_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3t/${v}_$r -o run -- python3 tests/perf/orb_bench.py 32 > gpurun_out/r3t/${v}_$r.log 2>&1 || exit 1
    python3 - gpurun_out/r3t/${v}_$r $v <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "orb_" in r["Name"]:
            print(sys.argv[2], r["Name"].split("(")[0].split("::")[-1], round(float(r["AverageNs"]) / 1000, 1), "us")
PY
  done
done
