set -o pipefail
# Round 5: the bench with its cfg2 side leg (ratio rule), the bench GPU tests.
OUT=gpurun_out/q6x; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bench.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().splitlines()[-1]); s=d['stages']; print(d['value'], d['ms_per_step'], d['roofline']['frac'], s['match_ms'], s['ransac_ms'], d['graph_checksum']); print('cfg2', d.get('cfg2')); c=d['cfg5']; print('cfg5', c.get('error'), c.get('s_per_reconstruction')); print('cfg3', d['cfg3']['match_ms'], d['cfg3']['k1_roofline']['frac'])"
