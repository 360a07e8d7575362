set -o pipefail
# A/B of the mutual kernel's column merge: atomics into one row per pair (default) vs per-query-
# block partials (SFM_MU_COLPART=1), interleaved bench runs on one box; then the K1 parity tests.
mkdir -p gpurun_out/colab
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_host.py -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/colab/pytest.log 2>&1 || { tail -20 gpurun_out/colab/pytest.log; exit 1; }
tail -1 gpurun_out/colab/pytest.log
for i in 1 2; do
  for v in 0 1; do
    SFM_MU_COLPART=$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/colab/bench_${v}_$i.json 2> gpurun_out/colab/bench_err_${v}_$i.txt || { tail -5 gpurun_out/colab/bench_err_${v}_$i.txt; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/colab/bench_${v}_$i.json')); print('colpart=$v', round(d['value']/1e6,2), round(d['ms_per_step'],2), 'K1', round(d['stages']['match_ms'],2), 'cfg3', d.get('cfg3',{}).get('ms_per_step'), d['graph_checksum'])"
  done
done
