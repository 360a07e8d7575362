set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tests/perf/k1_time.py 2>&1 | grep "xc="
