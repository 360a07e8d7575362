#!/bin/bash
# Incremental SfM 500 x 4096: BA calls instrumented, then rocprofv3 kernel stats of the same run.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python tests/perf/incremental_ba_probe.py > gpurun_out/r4k_probe.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4k_prof -o r4k -- python3 tests/perf/incremental_ba_probe.py > gpurun_out/r4k_prof.log 2>&1
