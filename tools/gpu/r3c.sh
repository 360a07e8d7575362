#!/bin/bash
# LDS column transpose variant: parity (match tests on the variant library) + interleaved A/B timing.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
SFMCORE_LIB=$PWD/sfm-project_amd/lib/libsfmcore_ldst.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 tests/test_gpu_match.py tests/test_gpu_golden.py > gpurun_out/r3c_pytest.log 2>&1 && \
K1_ONLY_BENCH_RULE=1 tools/ab_k1.sh 3 base ldst > gpurun_out/r3c_cfg3.txt && \
K1_ONLY_BENCH_RULE=1 N_IMG=40 K=4096 tools/ab_k1.sh 2 base ldst > gpurun_out/r3c_k4096.txt
