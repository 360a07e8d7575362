#!/bin/bash
# BA solve geometry A/B after the u = W t change: lanes per point (SFM_BA_PG 4/8/16) and threads
# per camera block (SFM_BA_CC 128/256/512), tests/perf/ba_solve_bench.py at cfg5, two rounds.
set -o pipefail
mkdir -p gpurun_out/r4f
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for v in base pg4 pg16 cc128 cc512; do
    L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
    SFMCORE_LIB=$L timeout -k 10 300 python tests/perf/ba_solve_bench.py > gpurun_out/r4f/${v}_$r.json 2> gpurun_out/r4f/${v}_$r.err || exit 1
    python3 -c "
import json; d=json.loads(open('gpurun_out/r4f/${v}_$r.json').read().strip().splitlines()[-1])
print('$v', round(d['cg_iter_ms']*1e3,1), 'us/iter', round(d['setup_backsub_ms']*1e3,1), 'us setup', round(d['lm_step_ms'],3), 'ms LM', d['cg_iters_to_1e-6'])"
  done
done
