#!/bin/bash
# Incremental SfM 500 x 4096: PCG tolerance of the bundle adjustments A/B (wall, BA, quality).
set -o pipefail
mkdir -p gpurun_out/r5b
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 500 python tests/perf/incremental_cgtol_ab.py 1e-10 1e-2 1e-1 > gpurun_out/r5b/ab.jsonl 2> gpurun_out/r5b/ab.err || { tail -20 gpurun_out/r5b/ab.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r5b/ab.jsonl'):
    d=json.loads(l); print(d['cg_tol'], round(d['wall_s'],3), [ (b['n_obs'], b['lm_steps'], b['cg_total'], round(b['s'],3)) for b in d['ba']], d['registered'], d['points'], round(d['median_reproj_px'],4), round(d['max_centre_err_rel_radius'],6))
"
