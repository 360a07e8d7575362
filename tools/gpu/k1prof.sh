set -o pipefail
TAG=${1:-k1p}
mkdir -p gpurun_out/kp_$TAG
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kp_$TAG -o run --output-format csv -- python3 tests/perf/k1_time.py > gpurun_out/kp_$TAG/out.txt 2>&1
rc=$?
grep "xc=" gpurun_out/kp_$TAG/out.txt
python3 -c "
import csv
for r in list(csv.DictReader(open('gpurun_out/kp_$TAG/run_kernel_stats.csv')))[:14]: print(r['Name'][:70], r['Calls'], r['AverageNs'], r['Percentage'])"
exit $rc
