# Round 6: where cfg5's BA wall goes — a kernel trace of one cfg5 reconstruction, GPU idle gaps
# attributed to the kernel before them (tools/trace_gaps.py), for the BA kernels and for all.
set -o pipefail
O=gpurun_out/s14; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --config cfg5 --steps 1 --warmup 1 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().splitlines()[-1]); c=d['cfg5']; print(round(c['s_per_reconstruction'],4), c['ba_phase_s'], c['stage_s'])"
T=$(ls $O/prof/run_kernel_trace.csv)
python3 tools/trace_gaps.py $T '(ba_|bas_)' > $O/gaps_ba.txt && cat $O/gaps_ba.txt
python3 tools/trace_gaps.py $T > $O/gaps_all.txt && head -40 $O/gaps_all.txt
