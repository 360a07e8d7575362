#!/bin/bash
# ORB without the per-level candidate cap: ORB GPU tests + the 1080p ORB bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_orb.py > gpurun_out/r3i_pytest.log 2>&1 && \
timeout -k 10 300 python tests/perf/orb_bench.py > gpurun_out/r3i_orb_bench.json 2> gpurun_out/r3i_orb.err
