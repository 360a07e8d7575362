set -o pipefail
# GPU-box driver scripts (run through gpurun from the repo root, e.g. gpurun -- bash tools/gpu/run_all.sh TAG).
TAG=${1:-r1c}
mkdir -p gpurun_out/prof_$TAG
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && cat gpurun_out/bench_$TAG.json &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG/bench.json 2> gpurun_out/prof_$TAG/bench.err && python3 -c "
import csv,sys
for r in list(csv.DictReader(open('gpurun_out/prof_$TAG/run_kernel_stats.csv')))[:8]: print(r['Name'][:60], r['Calls'], r['AverageNs'], r['Percentage'])"
