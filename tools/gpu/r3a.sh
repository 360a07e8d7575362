#!/bin/bash
# Round 3, first call: K1 block-lifetime breakdown (clock build) at cfg3 and K=4096, base timing.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
SFMCORE_LIB=$PWD/sfm-project_amd/lib/libsfmcore_clock.so timeout -k 10 180 python tests/perf/k1_clock.py > gpurun_out/r3a_clock_cfg3.json && \
SFMCORE_LIB=$PWD/sfm-project_amd/lib/libsfmcore_clock.so N_IMG=40 K=4096 timeout -k 10 180 python tests/perf/k1_clock.py > gpurun_out/r3a_clock_k4096.json && \
K1_ONLY_BENCH_RULE=1 timeout -k 10 120 python tests/perf/k1_time.py > gpurun_out/r3a_k1_time.txt
