set -o pipefail
# ORB ablation traces: tools/gpu/orb_abl.sh v1 v2 ... (lib/libsfmcore_<v>.so; "base" = libsfmcore.so)
export TMPDIR=/tmp
for v in "$@"; do
  L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
  SFMCORE_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/oabl/$v -o run --output-format csv -- python3 tests/perf/orb_bench.py 32 > gpurun_out/oabl/$v.json 2>/dev/null || { echo "$v failed"; exit 1; }
done
