#!/bin/bash
# fp64 RANSAC mode + batched verify_pairs + templated f32 path: GPU tests, then a cfg3 bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_ransac.py tests/test_gpu_golden.py tests/test_gpu_host.py tests/test_gpu_ba_lm.py tests/test_gpu_fullsize.py > gpurun_out/r3g_pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --config cfg3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3g_bench_cfg3.json 2> gpurun_out/r3g_bench.err
