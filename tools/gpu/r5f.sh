#!/bin/bash
# Graph row writers staged through LDS (coalesced dword stores): graph GPU tests, expansion timing
# (previous library graphold vs this one), graph_rows_kernel time in a cfg4 bench under rocprofv3.
set -o pipefail
mkdir -p gpurun_out/r5f
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_host.py tests/test_gpu_bench.py::test_bench_two_ranks_same_graph > gpurun_out/r5f/pytest.log 2>&1 || { tail -40 gpurun_out/r5f/pytest.log; exit 1; }
tail -2 gpurun_out/r5f/pytest.log
for v in graphold base; do
  L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
  SFMCORE_LIB=$L timeout -k 10 300 python tests/perf/graph_expand_time.py 8 > gpurun_out/r5f/expand_$v.json || exit 1
  echo $v; cat gpurun_out/r5f/expand_$v.json
  SFMCORE_LIB=$L timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5f/$v-cfg4 -o run -- python3 bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline --no-fp64 --no-cfg3 > gpurun_out/r5f/$v-cfg4.json 2> gpurun_out/r5f/$v-cfg4.err || { tail -5 gpurun_out/r5f/$v-cfg4.err; exit 1; }
  grep graph_rows gpurun_out/r5f/$v-cfg4/run_kernel_stats.csv | cut -c1-40,200-400
done
