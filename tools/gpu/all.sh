set -o pipefail
# full GPU test suite, then the perf scripts named on the command line (each under its own limit)
TAG=${1:-all}; shift
mkdir -p gpurun_out/all_$TAG
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider -x --timeout 300 --timeout-method thread > gpurun_out/all_$TAG/pytest.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/all_$TAG/pytest.log | tail -8
[ $rc -eq 0 ] || exit $rc
for s in "$@"; do
  n=$(basename $s .py)
  timeout -k 10 300 python $s > gpurun_out/all_$TAG/$n.json 2> gpurun_out/all_$TAG/$n.err || { tail -5 gpurun_out/all_$TAG/$n.err; exit 1; }
  cat gpurun_out/all_$TAG/$n.json
done
