#!/bin/bash
# ransac_fit_kernel ablations at cfg4 (timing only): rocprofv3 kernel stats of one bench step per
# library variant (base, nofit = no 8-point fit, noprev = no preview).
set -o pipefail
OUT=gpurun_out/${1:-fit_abl}; mkdir -p $OUT
export TMPDIR=/tmp
for v in base nofit noprev; do
  L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
  SFMCORE_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$v -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-cfg3 > $OUT/$v.log 2>&1 || { tail -5 $OUT/$v.log; exit 1; }
  python3 -c "
import csv,glob,sys
f=glob.glob('$OUT/$v/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'ransac' in r['Name']: print('$v', r['Name'].split('(')[0][-40:], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg')
"
done
