#!/bin/bash
# Incremental SfM end to end after the round-3 BA solve changes: cfg3 and 500 x 4096.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python tests/perf/incremental_bench.py > gpurun_out/r4j_inc_cfg3.log 2>&1 && \
timeout -k 10 600 python tests/perf/incremental_bench.py 500 4096 > gpurun_out/r4j_inc_500.log 2>&1
