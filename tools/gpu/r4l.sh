#!/bin/bash
# BA point pass on long tracks: loop unrolling (1/2/4) and 32 lanes per point, on the incremental
# 500 x 4096 problem (tracks of ~37 observations) and on cfg5 (5 per point).
set -o pipefail
mkdir -p gpurun_out/r4l
export PYTHONUNBUFFERED=1
for v in base u2 u4 pg32 pg32u2; do
  L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
  SFMCORE_LIB=$L timeout -k 10 400 python tests/perf/incremental_ba_probe.py > gpurun_out/r4l/inc_$v.json 2> gpurun_out/r4l/inc_$v.err || exit 1
  SFMCORE_LIB=$L timeout -k 10 400 python tests/perf/ba_solve_bench.py > gpurun_out/r4l/cfg5_$v.json 2> gpurun_out/r4l/cfg5_$v.err || exit 1
  python3 -c "
import json
a=json.loads(open('gpurun_out/r4l/inc_$v.json').read().strip().splitlines()[-1])
b=json.loads(open('gpurun_out/r4l/cfg5_$v.json').read().strip().splitlines()[-1])
print('$v', 'incremental wall', round(a['wall'],3), 'BA', [round(x['s'],3) for x in a['ba']], 'cg', [x['cg_total'] for x in a['ba']], '| cfg5 cg_iter_us', round(b['cg_iter_ms']*1e3,1), 'lm_ms', round(b['lm_step_ms'],3))"
done
