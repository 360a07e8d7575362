set -o pipefail
# Round 4: after removing the rejected K1 knobs (pair-info prologue, 16-B row records, prefetch,
# VALU query constant): the match / golden / host / bench GPU tests, the default-flag 2-rank gloo
# bench (rank 0's fp64 side leg before the final barrier), and the cfg4 line.
OUT=gpurun_out/r6o; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_golden.py tests/test_gpu_host.py tests/test_gpu_bench.py -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/pytest.log | head -20
tail -1 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --device 0 --steps 1 --warmup 1 --no-cfg3 --no-cfg5 --no-cpu-baseline > $OUT/bench_n2.json 2> $OUT/bench_n2.err || { tail -20 $OUT/bench_n2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_n2.json').read().splitlines()[-1]); print(d['n_gpus'], d['graph_checksum'], 'k2_fp64' in d)"
timeout -k 10 300 python -u bench.py --no-cfg5 --no-cfg3 --no-cpu-baseline --no-fp64 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().splitlines()[-1]); s=d['stages']; print(d['value'], d['ms_per_step'], s['match_ms'], s['ransac_ms'], d['graph_checksum'])"
