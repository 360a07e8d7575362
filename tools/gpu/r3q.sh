#!/bin/bash
# BA solve: the point pass hands u_o = W_o t_p to the camera pass (no camera-major W copy):
# BA GPU tests, then the cfg5 solve bench on the previous library and on this one.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ba_sharded.py tests/test_gpu_ba_lm.py tests/test_gpu_ba.py tests/test_gpu_incremental.py > gpurun_out/r3q_pytest.log 2>&1 && \
SFMCORE_LIB=$PWD/sfm-project_amd/lib/libsfmcore_baprev.so timeout -k 10 400 python tests/perf/ba_solve_bench.py > gpurun_out/r3q_ba_prev.json 2> gpurun_out/r3q_ba_prev.err && \
timeout -k 10 400 python tests/perf/ba_solve_bench.py > gpurun_out/r3q_ba_new.json 2> gpurun_out/r3q_ba_new.err && \
SFMCORE_LIB=$PWD/sfm-project_amd/lib/libsfmcore_baprev.so timeout -k 10 400 python tests/perf/ba_solve_bench.py > gpurun_out/r3q_ba_prev2.json 2> gpurun_out/r3q_ba_prev2.err && \
timeout -k 10 400 python tests/perf/ba_solve_bench.py > gpurun_out/r3q_ba_new2.json 2> gpurun_out/r3q_ba_new2.err
