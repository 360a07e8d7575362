# Round 6: K3 chunked vs unchunked at cfg5's final-model size — event timing and one PMC pass per
# form ("chunked K3 within 5 % of the unchunked form, or a PMC record of why not").
set -o pipefail
O=gpurun_out/s11; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do timeout -k 10 120 python tests/perf/ba_jtj_time.py 500 258000 4 >> $O/jtj_time.jsonl || exit 1; done
cat $O/jtj_time.jsonl
for f in plain chunked; do
  for set in "GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" "GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM"; do
    n=$(echo $set | md5sum | cut -c1-6)
    BA_JTJ_ONLY=$f timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "ba_" -d $O/pmc_${f}_$n -o run --output-format csv -- python3 tests/perf/ba_jtj_time.py 500 258000 4 > $O/pmc_${f}_$n.log 2>&1 || { echo "pmc $f failed"; tail $O/pmc_${f}_$n.log; exit 1; }
  done
  echo "== $f" >> $O/pmc.txt
  python3 tools/pmc_summary.py "$O" > /dev/null
  for d in $O/pmc_${f}_*; do [ -d $d ] && python3 tools/pmc_summary.py $d >> $O/pmc.txt; done
done
cat $O/pmc.txt
BA_JTJ_ONLY=plain timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/prof_plain -o run --output-format csv -- python3 tests/perf/ba_jtj_time.py 500 258000 4 > /dev/null 2>&1 || exit 1
BA_JTJ_ONLY=chunked timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/prof_chunked -o run --output-format csv -- python3 tests/perf/ba_jtj_time.py 500 258000 4 > /dev/null 2>&1 || exit 1
for f in plain chunked; do python3 - $f <<'PY'
import csv, sys
f = sys.argv[1]
for r in csv.DictReader(open(f'gpurun_out/s11/prof_{f}/run_kernel_stats.csv')):
    if r['Name'].startswith(('ba_', 'void ba_', '(anonymous namespace)::ba_', 'void (anonymous namespace)::ba_')) or 'ba_' in r['Name'][:45]:
        print(f"  {f} {r['Name'][:60]:60s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:9.1f} us")
PY
done
