set -o pipefail
mkdir -p gpurun_out/fitab
for v in base nofit noprev; do
  L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
  SFMCORE_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fitab/$v -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/fitab/$v.txt 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/fitab/$v/run_kernel_stats.csv')):
    if 'ransac' in r['Name']: print('$v', r['Name'][:40], r['AverageNs'])"
done
