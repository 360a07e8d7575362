#!/bin/bash
# cfg3 K1 stage breakdown: rocprofv3 kernel trace (per dispatch) + stats of a cfg3 bench run.
set -o pipefail
mkdir -p gpurun_out/r5a
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5a/prof -o run -- python3 bench.py --config cfg3 --steps 10 --warmup 3 --no-cpu-baseline --no-fp64 > gpurun_out/r5a/bench.json 2> gpurun_out/r5a/bench.err || { tail -20 gpurun_out/r5a/bench.err; exit 1; }
tail -c 1500 gpurun_out/r5a/bench.json
