set -o pipefail
# Round 5: K3 unchunked vs chunk mode; camera-only / observation-only ablation builds (timing only).
OUT=gpurun_out/q5k; mkdir -p $OUT
export TMPDIR=/tmp
for v in base camonly obsonly; do
  L=""; [ $v != base ] && L=sfm-project_amd/lib/libsfmcore_$v.so
  for g in 1 8; do
    SFMCORE_LIB=$L SFM_BA_CKW=$g timeout -k 10 200 python -u tests/perf/ba_jtj_time.py > $OUT/$v.$g.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/$v.$g.json'));print('$v ckw=$g', round(d['jtj_ms']*1000,1), round(d['jtj_chunked_ms']*1000,1))"
  done
done
