#!/bin/bash
# ORB tile kernel: FAST candidates appended with one LDS atomic per wave (four ballots)
# instead of one per lane: ORB GPU tests, tile kernel time (32 images) vs the previous build, ORB bench.
set -o pipefail
mkdir -p gpurun_out/r4i
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_orb.py > gpurun_out/r4i_pytest.log 2>&1 || exit 1
for r in 1 2; do
  for v in orbprev base; do
    L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
    SFMCORE_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4i/${v}_$r -o run -- python3 tests/perf/orb_bench.py 32 > gpurun_out/r4i/${v}_$r.log 2>&1 || exit 1
    python3 tools/orb_kstats.py gpurun_out/r4i/${v}_$r $v
  done
done
timeout -k 10 300 python tests/perf/orb_bench.py > gpurun_out/r4i_orb_bench.json 2> gpurun_out/r4i_orb_bench.err
