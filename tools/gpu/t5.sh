set -o pipefail
# T-build group sizes at cfg5's final model (bench cfg5 leg only, short cfg4 step).
OUT=gpurun_out/t5; mkdir -p $OUT
timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 --no-cfg3 --no-fp64 --no-local --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().splitlines()[-1]); c=d['cfg5']; print(json.dumps(c, indent=1)[:6000])"
