set -o pipefail
TAG=${1:-ab}
shift
mkdir -p gpurun_out/kp_$TAG
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/pytest_match_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_match_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/ab_k1.sh 1 "$@" 2>&1 | tee gpurun_out/kp_$TAG/ab.txt || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kp_$TAG -o run --output-format csv -- python3 tests/perf/k1_time.py > gpurun_out/kp_$TAG/out.txt 2>&1 || exit 1
python3 -c "
import csv
for r in list(csv.DictReader(open('gpurun_out/kp_$TAG/run_kernel_stats.csv')))[:14]: print(r['Name'][:70], r['Calls'], r['AverageNs'], r['Percentage'])"
