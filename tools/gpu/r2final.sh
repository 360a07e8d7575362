set -o pipefail
# round-2 closing run: GPU suite, default bench, rocprof kernel stats of the bench, K3 + ORB benches
TAG=${1:-r2g}
mkdir -p gpurun_out/$TAG/prof
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider -x --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/$TAG/pytest_gpu.log; exit 1; }
grep -E "passed|failed" gpurun_out/$TAG/pytest_gpu.log | tail -1
timeout -k 10 600 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -5 gpurun_out/$TAG/bench.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-cfg3 > gpurun_out/$TAG/prof/bench.json 2> gpurun_out/$TAG/prof/bench.err || { tail -5 gpurun_out/$TAG/prof/bench.err; exit 1; }
timeout -k 10 200 python tests/perf/ba_bench.py > gpurun_out/$TAG/ba_cfg5.json 2>/dev/null || exit 1
timeout -k 10 200 python tests/perf/orb_bench.py > gpurun_out/$TAG/orb.json 2>/dev/null || exit 1
echo done
