#!/bin/bash
# Round-3 closing validation (second session, after the tracks and driver changes): every GPU test, smoke(), the default bench, and
# rocprofv3 kernel stats of a short bench run.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5j_pytest.log 2>&1 || { tail -30 gpurun_out/r5j_pytest.log; exit 1; }
tail -3 gpurun_out/r5j_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5j_smoke.log 2>&1 || { tail -20 gpurun_out/r5j_smoke.log; exit 1; }
tail -1 gpurun_out/r5j_smoke.log
timeout -k 10 900 python bench.py > gpurun_out/r5j_bench.json 2> gpurun_out/r5j_bench.err || { tail -20 gpurun_out/r5j_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r5j_bench.json').read().strip().splitlines()[-1]); print(d['value']/1e6, d['ms_per_step'], d['graph_checksum'], d['roofline']['frac'], d['cfg3']['value']/1e6, d['cfg3']['ms_per_step'], d['cpu_baseline']['inlier_parity_with_gpu'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5j_prof -o r5j -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fp64 > gpurun_out/r5j_prof_bench.json 2> gpurun_out/r5j_prof.err
