set -o pipefail
# Round 5: K3 chunk mode, camera waves per camera (SFM_BA_CKW) A/B at the cfg5 final-model size.
OUT=gpurun_out/q5j; mkdir -p $OUT
export TMPDIR=/tmp
for g in 1 2 8 1 2 8; do
  SFM_BA_CKW=$g timeout -k 10 200 python -u tests/perf/ba_jtj_time.py >> $OUT/ckw.jsonl 2>> $OUT/ckw.err || { tail -20 $OUT/ckw.err; exit 1; }
done
cat $OUT/ckw.jsonl
