set -o pipefail
# A/B: 1024-thread mutual finalize (ft1024), 32-match RANSAC preview (pv32): cfg4 bench interleaved
mkdir -p gpurun_out/k1v2ab
export TMPDIR=/tmp
for i in 1 2; do
  for v in base ft1024 pv32; do
    L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
    SFMCORE_LIB=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/k1v2ab/b_${v}_$i.json 2> gpurun_out/k1v2ab/e_${v}_$i.txt || { tail -5 gpurun_out/k1v2ab/e_${v}_$i.txt; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/k1v2ab/b_${v}_$i.json')); print('$v', round(d['value']/1e6,2), round(d['ms_per_step'],2), 'K1', round(d['stages']['match_ms'],2), 'cfg3 K1', round(d['cfg3']['match_ms'],3), 'K2', round(d['stages']['ransac_ms'],2), d['graph_checksum'])"
  done
done
