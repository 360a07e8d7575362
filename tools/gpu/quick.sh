set -o pipefail
# quick perf check: selected GPU tests, cfg3 + cfg4 bench lines (no CPU leg), rocprof kernel stats on cfg3
TAG=${1:-q}
K=${2:-ransac}
mkdir -p gpurun_out/prof_$TAG
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 300 --timeout-method thread -k "$K" > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config cfg3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench3_$TAG.json 2>/dev/null && python3 -c "
import json; d=json.load(open('gpurun_out/bench3_$TAG.json')); print('cfg3', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],3), 'ms', d['stages']['match_ms'], d['stages']['ransac_ms'])" &&
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cfg3 > gpurun_out/bench4_$TAG.json 2>/dev/null && python3 -c "
import json; d=json.load(open('gpurun_out/bench4_$TAG.json')); print('cfg4', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],3), 'ms', d['stages']['match_ms'], d['stages']['ransac_ms'], d['roofline']['frac'])" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --config cfg3 --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2>&1 && python3 -c "
import csv
for r in list(csv.DictReader(open('gpurun_out/prof_$TAG/run_kernel_stats.csv')))[:10]: print(r['Name'][:60], r['Calls'], r['AverageNs'], r['Percentage'])"
