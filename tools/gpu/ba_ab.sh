set -o pipefail
# interleaved A/B of K3 library variants on tests/perf/ba_bench.py: tools/gpu/ba_ab.sh ROUNDS v1 v2 ...
R=$1; shift
for r in $(seq $R); do
  for v in "$@"; do
    L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
    SFMCORE_LIB=$L timeout -k 10 120 python tests/perf/ba_bench.py 2>/dev/null | python3 -c "
import json,sys; d=json.load(sys.stdin); print('$v', round(d['ms']*1000,1), 'us', round(d['roofline']['frac'],3), 'U_rel', d['parity']['U_rel'])" || exit 1
  done
done
