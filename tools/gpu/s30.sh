# Round 6: the mutual rule through the ratio path (now with the scan units) against the mutual
# kernel, at cfg3 (50 x 2048, all pairs) and on the cfg4 shard (K = 4096), bit-identity checked.
set -o pipefail
O=gpurun_out/s30; mkdir -p $O
export TMPDIR=/tmp
N_IMG=50 K=2048 SHARD=0/1 ROUNDS=5 timeout -k 10 300 python tests/perf/k1_mutual_ab.py >> $O/mutual_fr.jsonl || exit 1
timeout -k 10 300 python tests/perf/k1_mutual_ab.py >> $O/mutual_fr.jsonl || exit 1
cat $O/mutual_fr.jsonl
