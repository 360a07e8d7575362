set -o pipefail
# Round 4: kernel trace of one cfg5 reconstruction (GPU busy vs wall in the LM steps).
OUT=gpurun_out/r6s; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --config cfg5 --steps 1 --warmup 1 > $OUT/cfg5.json 2> $OUT/cfg5.err || { tail -30 $OUT/cfg5.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/cfg5.json').read().splitlines()[-1]); c=d['cfg5']; print(d['ms_per_step'], c['stage_s'], c['ba_phase_s'])"
