set -o pipefail
# round-2 driver: GPU tests (optionally a -k filter), then the default bench (cfg4) and a cfg3 bench.
TAG=${1:-r2}
K=${2:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'OMP', os.environ.get('OMP_NUM_THREADS'))"
if [ -n "$K" ]; then KF="-k $K"; else KF=""; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider -x --timeout 300 --timeout-method thread $KF > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_gpu_$TAG.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$?
tail -3 gpurun_out/bench_$TAG.err; cat gpurun_out/bench_$TAG.json
exit $rc
