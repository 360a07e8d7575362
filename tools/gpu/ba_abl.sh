set -o pipefail
# K3 ablation traces: tools/gpu/ba_abl.sh v1 v2 ... (lib/libsfmcore_<v>.so; "base" = libsfmcore.so)
export TMPDIR=/tmp
for v in "$@"; do
  L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; [ $v = base ] && L=$PWD/sfm-project_amd/lib/libsfmcore.so
  SFMCORE_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/abl/$v -o run -- python3 tests/perf/ba_bench.py > gpurun_out/abl/$v.json 2>/dev/null || { echo "$v failed"; exit 1; }
done
