#!/bin/bash
# Default bench (cfg4 + cfg3 side + fp64 side + CPU baseline), then rocprofv3 kernel stats of it.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python bench.py > gpurun_out/r3h_bench.json 2> gpurun_out/r3h_bench.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r3h_prof -o r3h -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fp64 > gpurun_out/r3h_prof_bench.json 2> gpurun_out/r3h_prof.err
