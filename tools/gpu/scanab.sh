set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for v in "$@"; do
  L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
  SFMCORE_LIB=$L timeout -k 10 120 python tests/perf/l2fr_scan_time.py 2>&1 | grep "scan-only" || exit 1
done; done
