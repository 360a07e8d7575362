set -o pipefail
# rocprof kernel stats of the default bench + K3 and ORB benches (the tail of r2final.sh)
TAG=${1:-r2g}
mkdir -p gpurun_out/$TAG/prof
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-cfg3 > gpurun_out/$TAG/prof/bench.json 2> gpurun_out/$TAG/prof/bench.err || { tail -5 gpurun_out/$TAG/prof/bench.err; exit 1; }
timeout -k 10 200 python tests/perf/ba_bench.py > gpurun_out/$TAG/ba_cfg5.json 2>/dev/null || exit 1
timeout -k 10 200 python tests/perf/orb_bench.py > gpurun_out/$TAG/orb.json 2>/dev/null || exit 1
echo done
