set -o pipefail
# BA tests + K3 bench at cfg5 + rocprof kernel stats
TAG=${1:-ba}
mkdir -p gpurun_out/ba_$TAG
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 300 --timeout-method thread -k "ba or recon or incremental or fullsize or smoke" > gpurun_out/ba_$TAG/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/ba_$TAG/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tests/perf/ba_bench.py > gpurun_out/ba_$TAG/bench.json 2>/dev/null && cat gpurun_out/ba_$TAG/bench.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ba_$TAG -o run --output-format csv -- python3 tests/perf/ba_bench.py > /dev/null 2>&1 && python3 -c "
import csv
for r in list(csv.DictReader(open('gpurun_out/ba_$TAG/run_kernel_stats.csv')))[:8]: print(r['Name'][:60], r['Calls'], r['AverageNs'], r['Percentage'])"
