#!/bin/bash
# Executed share of K2 scoring on the cfg4 scene: VALU instructions of the pruned vs the unpruned
# score kernel over the same pair sample (tests/perf/ransac_exec_frac.py), one PMC pass.
set -o pipefail
TAG=${1:-pmc_ransac_exec}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "ransac_score" -d $OUT/p1 -o run --output-format csv -- python3 tests/perf/ransac_exec_frac.py > $OUT/p1.log 2>&1 || { echo "pass failed"; tail -5 $OUT/p1.log; exit 1; }
cat $OUT/p1.log | grep pairs=
python3 - $OUT <<'PY'
import csv, glob, re, sys, collections
acc = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + "/p1/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[(re.search(r"ransac_score_kernel<[^>]*>", r["Kernel_Name"]).group(0), r["Counter_Name"])] += float(r["Counter_Value"])
for k, v in sorted(acc.items()):
    print(k, f"{v:.6g}")
PY
