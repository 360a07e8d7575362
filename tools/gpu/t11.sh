set -o pipefail
# Round 6 validation (6, the closing tree with the staged T build): whole GPU suite, smoke(), the default bench line (cfg4 + calib + cfg3 / cfg2 /
# cfg4_local / cfg5 legs), rocprofv3 kernel stats of the bench (no cfg5 / local legs), and the
# cfg2 call under rocprofv3 (kernel stats) + one PMC pass of the ratio path's kernels.
OUT=gpurun_out/t11; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -30
tail -1 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().splitlines()[-1]); s=d['stages']; print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['frac_of_practical'], d['calib'], s['match_ms'], s['ransac_ms'], d['graph_checksum']); l=d.get('cfg4_local', {}); print('local', l.get('error'), l.get('value'), l.get('match_ms'), l.get('ransac_ms')); c=d['cfg5']; print('cfg5', c.get('error'), c.get('value'), c.get('s_per_reconstruction'), c.get('points'), c.get('ba_phase_s')); print('cfg3', d['cfg3']['match_ms'], d['cfg3']['k1_roofline']['frac']); print('cfg2', d['cfg2'])"
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cfg5 --no-local > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -30 $OUT/bench_prof.err; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/prof_cfg2 -o run --output-format csv -- python3 tests/perf/k1_cfg2_time.py ratio > $OUT/prof_cfg2.log 2>&1 || { tail $OUT/prof_cfg2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-include-regex "l2fr_" -d $OUT/pmc_cfg2 -o run --output-format csv -- python3 tests/perf/k1_cfg2_time.py ratio > $OUT/pmc_cfg2.log 2>&1 || { tail $OUT/pmc_cfg2.log; exit 1; }
python3 tools/pmc_summary.py $OUT/pmc_cfg2 > $OUT/pmc_cfg2.txt && cat $OUT/pmc_cfg2.txt
find $OUT/prof $OUT/prof_cfg2 -name "*kernel_stats.csv"
