set -o pipefail
# A/B of the mutual kernel's row records: 8 B (default) vs 16 B (libsfmcore_rowi4.so), cfg4 bench
# interleaved on one box, after the K1 parity tests on the default library.
mkdir -p gpurun_out/rowab
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_host.py -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/rowab/pytest.log 2>&1 || { tail -20 gpurun_out/rowab/pytest.log; exit 1; }
tail -1 gpurun_out/rowab/pytest.log
for i in 1 2; do
  for v in base rowi4; do
    L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
    SFMCORE_LIB=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rowab/b_${v}_$i.json 2> gpurun_out/rowab/e_${v}_$i.txt || { tail -5 gpurun_out/rowab/e_${v}_$i.txt; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/rowab/b_${v}_$i.json')); print('$v', round(d['value']/1e6,2), round(d['ms_per_step'],2), 'K1', round(d['stages']['match_ms'],2), 'cfg3', round(d['cfg3']['ms_per_step'],3), d['graph_checksum'])"
  done
done
