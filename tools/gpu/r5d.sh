#!/bin/bash
# Graph exchange: kernel-written packed rows + one-launch expansion (sfm_graph_expand): the graph /
# all-gather GPU tests, the two-rank bench rehearsal, the sharded incremental driver, and the
# expansion timing at cfg4 size (8 ranks' gathered layout).
set -o pipefail
mkdir -p gpurun_out/r5d
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_host.py tests/test_gpu_bench.py tests/test_gpu_fullsize.py::test_rccl_world1_graph_allgather_and_camera_allreduce tests/test_gpu_incremental.py::test_incremental_sharded_matching_two_ranks > gpurun_out/r5d/pytest.log 2>&1 || { tail -40 gpurun_out/r5d/pytest.log; exit 1; }
tail -5 gpurun_out/r5d/pytest.log
timeout -k 10 300 python tests/perf/graph_expand_time.py 8 > gpurun_out/r5d/expand8.json && timeout -k 10 300 python tests/perf/graph_expand_time.py 2 > gpurun_out/r5d/expand2.json && cat gpurun_out/r5d/expand8.json gpurun_out/r5d/expand2.json
