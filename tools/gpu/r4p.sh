#!/bin/bash
# BA camera pass: four observations' gathers in flight per lane. BA GPU tests, bit check against
# the previous build, cfg5 solve bench interleaved (2 rounds), kernel split from the shard probe.
set -o pipefail
mkdir -p gpurun_out/r4p
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_ba_lm.py tests/test_gpu_ba_sharded.py > gpurun_out/r4p_pytest.log 2>&1 || { tail -20 gpurun_out/r4p_pytest.log; exit 1; }
SFMCORE_LIB=$PWD/sfm-project_amd/lib/libsfmcore_baprev.so timeout -k 10 200 python tests/perf/ba_bits.py gpurun_out/r4p/bits_prev.npz && \
timeout -k 10 200 python tests/perf/ba_bits.py gpurun_out/r4p/bits_new.npz || exit 1
for r in 1 2; do
  for v in baprev base; do
    L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
    SFMCORE_LIB=$L timeout -k 10 300 python tests/perf/ba_solve_bench.py > gpurun_out/r4p/${v}_$r.json 2> gpurun_out/r4p/${v}_$r.err || exit 1
    python3 -c "
import json; d=json.loads(open('gpurun_out/r4p/${v}_$r.json').read().strip().splitlines()[-1])
print('$v', round(d['cg_iter_ms']*1e3,1), 'us/iter', round(d['lm_step_ms'],3), 'ms LM', round(d['sharded_world1_rccl']['cg_iter_ms']*1e3,1), 'us sharded')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4p/prof -o run -- python3 tests/perf/ba_shard_probe.py > gpurun_out/r4p/prof.log 2>&1
