#!/bin/bash
# Interleaved A/B of K1/K2 library variants (lib/libsfmcore_<v>.so, base = the default library): K2 ms
# of the cfg4 bench step and the cfg3 launch (tests/perf/ransac_variants.py, parity on a sample).
# Usage: tools/gpu/ransac_lib_ab.sh TAG ROUNDS v1 v2 ...
set -o pipefail
OUT=gpurun_out/$1; R=$2; shift 2; mkdir -p $OUT
for r in $(seq $R); do
  for v in "$@"; do
    L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
    SFMCORE_LIB=$L timeout -k 10 240 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-cfg3 > $OUT/cfg4_${v}_r$r.json 2> $OUT/cfg4_${v}_r$r.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('cfg4', sys.argv[2], 'match_ms %.3f' % d['stages']['match_ms'], 'ransac_ms %.3f' % d['stages']['ransac_ms'], 'step_ms %.2f' % d['ms_per_step'], 'verified %d' % d['verified_matches_per_step'])" $OUT/cfg4_${v}_r$r.json $v | tee -a $OUT/summary.txt
    SFMCORE_LIB=$L MODES=0 timeout -k 10 200 python3 tests/perf/ransac_variants.py 2>/dev/null | sed "s/^/cfg3 $v /" | tee -a $OUT/summary.txt || exit 1
  done
done
