set -o pipefail
# A/B of library variants (tools/build_variant.sh) on the full bench step: the K1/K2 parity tests
# against each non-base variant, then a rocprofv3 kernel trace of bench.py per variant.
# Usage (through gpurun, from the repo root): bash tools/gpu/varab.sh TAG base name1 ...
TAG=$1; shift
OUT=gpurun_out/varab_$TAG; mkdir -p $OUT
export TMPDIR=/tmp
lib() { if [ $1 = base ]; then echo $PWD/sfm-project_amd/lib/libsfmcore.so; else echo $PWD/sfm-project_amd/lib/libsfmcore_$1.so; fi; }
for v in "$@"; do
  [ $v = base ] && continue
  SFMCORE_LIB=$(lib $v) timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_ransac.py tests/test_gpu_golden.py -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > $OUT/pytest_$v.log 2>&1 || { tail -20 $OUT/pytest_$v.log; exit 1; }
  echo "$v tests: $(tail -1 $OUT/pytest_$v.log)"
done
for v in "$@"; do
  SFMCORE_LIB=$(lib $v) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$v -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/$v.json 2> $OUT/$v.err || exit 1
  python3 - "$OUT" "$v" <<'PY'
import csv, json, sys
out, v = sys.argv[1], sys.argv[2]
b = json.loads(open(f"{out}/{v}.json").read().strip().splitlines()[-1])
print(v, "ms/step %.4f" % b["ms_per_step"], "ransac %.4f" % b["stages"]["ransac_ms"])
for r in csv.DictReader(open(f"{out}/{v}/run_kernel_stats.csv")):
    if "ransac" in r["Name"]:
        print("   ", r["Name"][:44], r["AverageNs"])
PY
done
