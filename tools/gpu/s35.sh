# Round 6: what the mutual kernel's block-end column merge (4096 u64 atomicMax per block at
# K = 4096) costs: the timing-only -DMU_DIAG_NOMERGE build (wrong results) against the default, on
# the cfg4 shard (tests/perf/k1_mutual_ab.py's mutual timings), interleaved.
set -o pipefail
O=gpurun_out/s35; mkdir -p $O
export TMPDIR=/tmp
NM=$PWD/sfm-project_amd/lib/libsfmcore_nomerge.so
for r in 1 2; do
  ROUNDS=2 timeout -k 10 300 python tests/perf/k1_mutual_ab.py | sed 's/^/base /' >> $O/merge_ab.txt || exit 1
  SFMCORE_LIB=$NM ROUNDS=2 timeout -k 10 300 python tests/perf/k1_mutual_ab.py | sed 's/^/nomerge /' >> $O/merge_ab.txt || exit 1
done
python3 -c "
import json
for l in open('$O/merge_ab.txt'):
    tag, js = l.split(' ', 1); d = json.loads(js); print(tag, [round(x, 2) for x in d['ms_mutual']])"
