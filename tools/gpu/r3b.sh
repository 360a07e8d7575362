#!/bin/bash
# K1 query-tiles-per-wave A/B (cfg3 and K=4096), interleaved, bench rule only.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 K1_ONLY_BENCH_RULE=1
tools/ab_k1.sh 3 base qt8w1 qt8w1c32 qt6 qt4w1 > gpurun_out/r3b_cfg3.txt && \
N_IMG=40 K=4096 tools/ab_k1.sh 2 base qt8w1 qt8w1c32 qt6 > gpurun_out/r3b_k4096.txt
