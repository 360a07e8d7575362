set -o pipefail
# Round 4: K2 preview length A/B (RANSAC_PV 64 = base vs 32 / 96 / 128; results are exact either
# way — the preview only orders the hypotheses), cfg4 bench, interleaved, two rounds.
OUT=gpurun_out/r6i; mkdir -p $OUT
for r in 1 2; do
  for v in base pv32 pv96 pv128; do
    L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
    SFMCORE_LIB=$L timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cfg3 --no-cfg5 --no-fp64 > $OUT/$v.$r.json 2> $OUT/$v.$r.err || { tail -5 $OUT/$v.$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/$v.$r.json').read().splitlines()[-1]); print('$v', $r, round(d['ms_per_step'],2), round(d['stages']['ransac_ms'],2), round(d['stages']['match_ms'],2), d['graph_checksum'])"
  done
done
