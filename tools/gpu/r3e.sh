#!/bin/bash
# Round 3: rank-2 spec change + skimage pins + RANSAC stats: the RANSAC / golden / match GPU tests.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_golden.py tests/test_gpu_ransac.py tests/test_gpu_match.py > gpurun_out/r3e_pytest.log 2>&1
