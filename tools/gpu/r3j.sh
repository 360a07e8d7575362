#!/bin/bash
# Sharded BA: one-launch finish (bas_pcg_finish_vec): BA GPU tests + the cfg5 solve bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ba_sharded.py tests/test_gpu_ba_lm.py tests/test_gpu_ba.py > gpurun_out/r3j_pytest.log 2>&1 && \
timeout -k 10 400 python tests/perf/ba_solve_bench.py > gpurun_out/r3j_ba_bench.json 2> gpurun_out/r3j_ba.err
