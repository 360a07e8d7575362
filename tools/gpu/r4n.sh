#!/bin/bash
# BA point pass: long tracks (> 64 observations) by a wave per point in extra blocks: BA +
# incremental GPU tests, the incremental 500 x 4096 probe and bench, and the cfg5 solve bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_ba_lm.py tests/test_gpu_ba_sharded.py tests/test_gpu_incremental.py > gpurun_out/r4n_pytest.log 2>&1 || { tail -20 gpurun_out/r4n_pytest.log; exit 1; }
timeout -k 10 400 python tests/perf/incremental_ba_probe.py > gpurun_out/r4n_probe.json 2> gpurun_out/r4n_probe.err && \
timeout -k 10 400 python tests/perf/incremental_bench.py 500 4096 > gpurun_out/r4n_inc_500.log 2>&1 && \
timeout -k 10 400 python tests/perf/incremental_bench.py > gpurun_out/r4n_inc_cfg3.log 2>&1 && \
timeout -k 10 400 python tests/perf/ba_solve_bench.py > gpurun_out/r4n_ba_cfg5.json 2> gpurun_out/r4n_ba_cfg5.err
