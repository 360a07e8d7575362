set -o pipefail
# rocprofv3 kernel stats of the default (cfg4) bench, one timed step
TAG=${1:-p4}
mkdir -p gpurun_out/prof4_$TAG
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4_$TAG -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-cfg3 > gpurun_out/prof4_$TAG/bench.json 2> gpurun_out/prof4_$TAG/bench.err && python3 -c "
import csv
for r in list(csv.DictReader(open('gpurun_out/prof4_$TAG/run_kernel_stats.csv')))[:14]: print(r['Name'][:60], r['Calls'], r['AverageNs'], r['TotalDurationNs'], r['Percentage'])"
