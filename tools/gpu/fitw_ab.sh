set -o pipefail
# A/B of the RANSAC fit kernel occupancy (RANSAC_FIT_MINW build knob): cfg4 bench interleaved
mkdir -p gpurun_out/fwab
export TMPDIR=/tmp
for i in 1 2; do
  for v in base fw6 fw8; do
    L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
    SFMCORE_LIB=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/fwab/b_${v}_$i.json 2> gpurun_out/fwab/e_${v}_$i.txt || { tail -5 gpurun_out/fwab/e_${v}_$i.txt; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/fwab/b_${v}_$i.json')); print('$v', round(d['value']/1e6,2), round(d['ms_per_step'],2), 'K2', round(d['stages']['ransac_ms'],2), 'cfg3 K2', round(d['cfg3']['ransac_ms'],3), d['graph_checksum'])"
  done
done
