#!/bin/bash
# K1 candidate bounds (timing only, wrong results by construction): column key build free (nokey),
# no block-end column merge (nomerge), interleaved with the shipped kernel.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
K1_ONLY_BENCH_RULE=1 tools/ab_k1.sh 3 base nokey nomerge > gpurun_out/r3p_cfg3.txt && \
K1_ONLY_BENCH_RULE=1 N_IMG=40 K=4096 tools/ab_k1.sh 2 base nokey nomerge > gpurun_out/r3p_k4096.txt
