set -o pipefail
# Round 4: K2 preview length A/B, second pass (64 = base, 128, 160, 192, 224) at cfg4 and cfg3.
OUT=gpurun_out/r6j; mkdir -p $OUT
for r in 1 2; do
  for v in base pv128 pv160 pv192 pv224; do
    L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
    for c in cfg4 cfg3; do
      SFMCORE_LIB=$L timeout -k 10 200 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-cfg3 --no-cfg5 --no-fp64 > $OUT/$v.$c.$r.json 2> $OUT/$v.$c.$r.err || { tail -5 $OUT/$v.$c.$r.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/$v.$c.$r.json').read().splitlines()[-1]); print('$v', '$c', $r, round(d['ms_per_step'],3), round(d['stages']['ransac_ms'],3), d['graph_checksum'])"
    done
  done
done
