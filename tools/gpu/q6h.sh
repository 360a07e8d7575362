set -o pipefail
# Round 5: host-side cProfile of one cfg5 reconstruction.
OUT=gpurun_out/q6h; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u tests/perf/recon_host_profile.py > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
grep -c . $OUT/prof.log
