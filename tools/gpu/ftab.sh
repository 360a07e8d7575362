set -o pipefail
mkdir -p gpurun_out/ftab
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/ftab/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/ftab/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in base; do
  L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
  SFMCORE_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ftab/$v -o run --output-format csv -- python3 tests/perf/k1_time.py > gpurun_out/ftab/$v.txt 2>&1 || exit 1
  grep "path=mutual" gpurun_out/ftab/$v.txt | head -1 | sed "s/^/$v /"
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/ftab/$v/run_kernel_stats.csv')):
    if 'mutual' in r['Name'] or 'pair_order' in r['Name'] or 'prep' in r['Name']: print('   ', r['Name'][:50], r['AverageNs'])"
done
