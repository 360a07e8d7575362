#!/bin/bash
# Incremental SfM 500 x 4096 after the driver changes; cfg4 two-rank gloo rehearsal of the bench's
# N > 1 step (packed rows + sfm_graph_expand) on one GPU: same graph checksum as N = 1.
set -o pipefail
mkdir -p gpurun_out/r5h
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python tests/perf/incremental_bench.py 500 4096 > gpurun_out/r5h/inc1.json 2> gpurun_out/r5h/inc1.err || { tail -20 gpurun_out/r5h/inc1.err; exit 1; }
timeout -k 10 300 python tests/perf/incremental_bench.py 500 4096 > gpurun_out/r5h/inc2.json 2> gpurun_out/r5h/inc2.err || { tail -20 gpurun_out/r5h/inc2.err; exit 1; }
python3 -c "
import json
for f in ('inc1','inc2'):
    d=json.loads(open('gpurun_out/r5h/'+f+'.json').read().strip().splitlines()[-1]); print(f, round(d['wall_s'],3), d['stage_s'], d['registered'], d['points'], round(d['median_reproj_px'],4))"
OMP_NUM_THREADS=8 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --no-fp64 --dist-backend gloo --device 0 > gpurun_out/r5h/bench_n2_gloo.json 2> gpurun_out/r5h/bench_n2_gloo.err || { tail -20 gpurun_out/r5h/bench_n2_gloo.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r5h/bench_n2_gloo.json').read().strip().splitlines()[-1]); print('n2 gloo same GPU', d['verified_matches_per_step'], d['graph_checksum'], d['ms_per_step'], d['stages'])"
