#!/bin/bash
# PMC passes over tests/perf/orb_bench.py for the ORB kernels (one counter group per pass).
set -o pipefail
TAG=${1:-pmc_orb}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "orb_" -d $OUT/p$i -o run --output-format csv -- python3 tests/perf/orb_bench.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, re, sys, collections
acc = collections.defaultdict(float); nd = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = re.search(r"orb_\w+", r["Kernel_Name"]).group(0)
        acc[(k, r["Counter_Name"])] += float(r["Counter_Value"]); nd[k].add(r["Dispatch_Id"])
for (k, c), v in sorted(acc.items()):
    print(f"{k:20s} {c:22s} {v / len(nd[k]):.4g}  (per dispatch, {len(nd[k])} dispatches)")
PY
