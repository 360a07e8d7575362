set -o pipefail
# Round 4: interleaved A/B, the K1 knob cleanup (base) against the previous source (prev), cfg4.
OUT=gpurun_out/r6p; mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in base prev; do
    L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
    SFMCORE_LIB=$L timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cfg3 --no-cfg5 --no-fp64 > $OUT/cfg4_${v}_r$r.json 2> $OUT/cfg4_${v}_r$r.err || { tail -20 $OUT/cfg4_${v}_r$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], 'match_ms %.2f' % d['stages']['match_ms'], 'ransac_ms %.2f' % d['stages']['ransac_ms'], 'step_ms %.2f' % d['ms_per_step'], d['graph_checksum'])" $OUT/cfg4_${v}_r$r.json $v $r
  done
done
