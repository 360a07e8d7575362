#!/bin/bash
# Sharded BA: camera phase 3 leaves U_d p, finish reads 24 doubles per camera: tests, probe, trace, solve bench.
set -o pipefail
mkdir -p gpurun_out/r3o
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ba_sharded.py tests/test_gpu_ba_lm.py > gpurun_out/r3o_pytest.log 2>&1 && \
timeout -k 10 300 python tests/perf/ba_shard_probe.py > gpurun_out/r3o_probe.json 2> gpurun_out/r3o_probe.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3o/prof -o run -- python tests/perf/ba_shard_probe.py > gpurun_out/r3o_prof.log 2>&1 && \
timeout -k 10 400 python tests/perf/ba_solve_bench.py > gpurun_out/r3o_ba_bench.json 2> gpurun_out/r3o_ba.err
