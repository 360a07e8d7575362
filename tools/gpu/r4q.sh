#!/bin/bash
# Round-3 validation: every GPU test, smoke(), the default bench, and rocprofv3 kernel stats of a
# short bench run (CSV) for profiles/r03.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4q_pytest.log 2>&1 || { tail -30 gpurun_out/r4q_pytest.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4q_smoke.log 2>&1 || { tail -20 gpurun_out/r4q_smoke.log; exit 1; }
timeout -k 10 900 python bench.py > gpurun_out/r4q_bench.json 2> gpurun_out/r4q_bench.err || { tail -20 gpurun_out/r4q_bench.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4q_prof -o r4q -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fp64 > gpurun_out/r4q_prof_bench.json 2> gpurun_out/r4q_prof.err
