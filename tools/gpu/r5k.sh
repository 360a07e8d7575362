#!/bin/bash
# RANSAC order kernel: per-wave histograms + parallel bucket offsets (base) vs the single-thread
# offset chain (ordold): RANSAC GPU tests, then kernel stats of cfg3 and cfg4 bench runs for both.
set -o pipefail
mkdir -p gpurun_out/r5k
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_ransac.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py::test_cfg3_full_launch_every_pair tests/test_gpu_fullsize.py::test_cfg4_shard_sample tests/test_gpu_bench.py > gpurun_out/r5k/pytest.log 2>&1 || { tail -40 gpurun_out/r5k/pytest.log; exit 1; }
tail -2 gpurun_out/r5k/pytest.log
for v in ordold base; do
  L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
  for c in cfg3 cfg4; do
    S=10; [ $c = cfg4 ] && S=2
    SFMCORE_LIB=$L timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5k/$v-$c -o run -- python3 bench.py --config $c --steps $S --warmup 1 --no-cpu-baseline --no-fp64 --no-cfg3 > gpurun_out/r5k/$v-$c.json 2> gpurun_out/r5k/$v-$c.err || { tail -5 gpurun_out/r5k/$v-$c.err; exit 1; }
    python3 -c "
import json,csv; d=json.loads(open('gpurun_out/r5k/$v-$c.json').read().strip().splitlines()[-1])
o=[x for x in csv.DictReader(open('gpurun_out/r5k/$v-$c/run_kernel_stats.csv')) if 'ransac_order' in x['Name'] or 'ransac_score' in x['Name']]
print('$v $c', round(d['value']/1e6,2), round(d['ms_per_step'],3), d['graph_checksum'], round(d['stages']['ransac_roofline']['executed_frac'],4), [(x['Name'][:30], round(float(x['AverageNs'])/1e3,1)) for x in o])"
  done
done
