#!/bin/bash
# ransac_stats_kernel grid-stride (three atomics per block): RANSAC / bench GPU tests, then
# rocprofv3 kernel stats of a short bench run.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_ransac.py tests/test_gpu_bench.py tests/test_gpu_fullsize.py > gpurun_out/r4g_pytest.log 2>&1 || { tail -20 gpurun_out/r4g_pytest.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4g_prof -o r4g -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fp64 > gpurun_out/r4g_prof_bench.json 2> gpurun_out/r4g_prof.err
