set -o pipefail
TAG=${1:-k1}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/pytest_match_$TAG.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_match_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tests/perf/k1_time.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/k1_time_$TAG.txt
