# Round 6: host-side profile of one cfg5 reconstruction (cProfile), for the BA set-up phase.
set -o pipefail
O=gpurun_out/s28; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python tests/perf/cfg5_host_profile.py 60 > $O/profile.txt 2> $O/profile.err || { tail -20 $O/profile.err; exit 1; }
head -3 $O/profile.txt
