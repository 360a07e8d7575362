#!/bin/bash
# Persistent K1 schedule: parity tests, interleaved A/B against the per-item grid, clock breakdown.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 tests/test_gpu_match.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py tests/test_gpu_host.py > gpurun_out/r3d_pytest.log 2>&1 && \
for r in 1 2 3; do for v in 0 1; do SFM_MU_PERSIST=$v K1_ONLY_BENCH_RULE=1 timeout -k 10 120 python tests/perf/k1_time.py | sed "s/^/persist=$v /"; done; done > gpurun_out/r3d_cfg3.txt && \
for r in 1 2; do for v in 0 1; do SFM_MU_PERSIST=$v N_IMG=40 K=4096 K1_ONLY_BENCH_RULE=1 timeout -k 10 120 python tests/perf/k1_time.py | sed "s/^/persist=$v /"; done; done > gpurun_out/r3d_k4096.txt && \
SFMCORE_LIB=$PWD/sfm-project_amd/lib/libsfmcore_clock.so timeout -k 10 180 python tests/perf/k1_clock.py > gpurun_out/r3d_clock_cfg3.json
