#!/bin/bash
# BA PCG: u_o stored at the observation's camera-major slot (the camera pass reads its rows
# contiguously instead of gathering through cam_obs).  BA GPU tests, bit comparison against the
# previous build (baold), cfg5 solve bench interleaved (2 rounds), incremental GPU tests.
set -o pipefail
mkdir -p gpurun_out/r5o
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_ba_lm.py tests/test_gpu_ba_sharded.py tests/test_gpu_incremental.py > gpurun_out/r5o/pytest.log 2>&1 || { tail -30 gpurun_out/r5o/pytest.log; exit 1; }
tail -2 gpurun_out/r5o/pytest.log
SFMCORE_LIB=$PWD/sfm-project_amd/lib/libsfmcore_baold.so timeout -k 10 200 python tests/perf/ba_bits.py gpurun_out/r5o/bits_old.npz && \
timeout -k 10 200 python tests/perf/ba_bits.py gpurun_out/r5o/bits_new.npz || exit 1
python3 -c "
import numpy as np
a=np.load('gpurun_out/r5o/bits_old.npz'); b=np.load('gpurun_out/r5o/bits_new.npz')
print('bit-identical:', all(np.array_equal(a[k], b[k]) for k in a.files), a.files)"
for r in 1 2; do
  for v in baold base; do
    L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
    SFMCORE_LIB=$L timeout -k 10 300 python tests/perf/ba_solve_bench.py > gpurun_out/r5o/${v}_$r.json 2> gpurun_out/r5o/${v}_$r.err || exit 1
    python3 -c "
import json; d=json.loads(open('gpurun_out/r5o/${v}_$r.json').read().strip().splitlines()[-1])
print('$v', round(d['cg_iter_ms']*1e3,1), 'us/iter', round(d['lm_step_ms'],3), 'ms LM', round(d['default_lm_step']['ms_poll_every_8'],3), 'ms default LM', round(d['sharded_world1_rccl']['cg_iter_ms']*1e3,1), 'us sharded')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5o/prof -o run -- python3 tests/perf/ba_shard_probe.py > gpurun_out/r5o/prof.log 2>&1
