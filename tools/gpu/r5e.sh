#!/bin/bash
# RANSAC prep kernel with four waves per pair: RANSAC parity tests, then kernel stats of cfg3 and
# cfg4 bench runs for the previous library (prepold) and this one.
set -o pipefail
mkdir -p gpurun_out/r5e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_ransac.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py::test_cfg3_full_launch_every_pair tests/test_gpu_fullsize.py::test_cfg4_shard_sample tests/test_gpu_fullsize.py::test_ransac_f64_mode_full_size > gpurun_out/r5e/pytest.log 2>&1 || { tail -40 gpurun_out/r5e/pytest.log; exit 1; }
tail -3 gpurun_out/r5e/pytest.log
for v in prepold base; do
  L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
  for c in cfg3 cfg4; do
    S=10; [ $c = cfg4 ] && S=2
    SFMCORE_LIB=$L timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5e/$v-$c -o run -- python3 bench.py --config $c --steps $S --warmup 1 --no-cpu-baseline --no-fp64 --no-cfg3 > gpurun_out/r5e/$v-$c.json 2> gpurun_out/r5e/$v-$c.err || { tail -5 gpurun_out/r5e/$v-$c.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r5e/$v-$c.json').read().strip().splitlines()[-1]); print('$v $c', d['value']/1e6, d['ms_per_step'], d['graph_checksum'])"
  done
done
