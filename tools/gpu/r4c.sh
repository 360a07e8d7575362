#!/bin/bash
# ORB select kernel: orientation / descriptor loads issued together (disk table, reciprocal root
# per keypoint), 512-thread blocks (1024 spills): ORB GPU tests, then the select kernel time
# (rocprofv3 stats, 32 images) for the previous build, this one and the 1024-thread variant.
set -o pipefail
mkdir -p gpurun_out/r4c
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_orb.py > gpurun_out/r4c_pytest.log 2>&1 || exit 1
for r in 1 2; do
  for v in orbprev base sel1024; do
    L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
    SFMCORE_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4c/${v}_$r -o run -- python3 tests/perf/orb_bench.py 32 > gpurun_out/r4c/${v}_$r.log 2>&1 || exit 1
    python3 tools/orb_kstats.py gpurun_out/r4c/${v}_$r $v
  done
done
timeout -k 10 300 python tests/perf/orb_bench.py > gpurun_out/r4c_orb_bench.json 2> gpurun_out/r4c_orb_bench.err
