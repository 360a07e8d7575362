#!/bin/bash
# Incremental driver with the inexact-Newton PCG default (ba_cg_tol 0.1): its GPU tests and the
# 500 x 4096 bench.
set -o pipefail
mkdir -p gpurun_out/r5c
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_incremental.py > gpurun_out/r5c/pytest.log 2>&1 || { tail -30 gpurun_out/r5c/pytest.log; exit 1; }
tail -8 gpurun_out/r5c/pytest.log
timeout -k 10 300 python tests/perf/incremental_bench.py 500 4096 > gpurun_out/r5c/inc.json 2> gpurun_out/r5c/inc.err || { tail -20 gpurun_out/r5c/inc.err; exit 1; }
tail -c 900 gpurun_out/r5c/inc.json
