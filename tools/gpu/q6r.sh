set -o pipefail
# Round 5: P3P scoring with a hypothesis' poses interleaved (REG_INTERLEAVE=1, lib variant regil)
# against the default: registration parity tests on the variant, then reg_hyp_kernel time in the
# cfg5 leg, interleaved A/B (rocprofv3 kernel stats).
OUT=gpurun_out/q6r; mkdir -p $OUT
export TMPDIR=/tmp
SFMCORE_LIB=$PWD/sfm-project_amd/lib/libsfmcore_regil.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_register.py > $OUT/pytest_regil.log 2>&1 || { tail -30 $OUT/pytest_regil.log; exit 1; }
tail -1 $OUT/pytest_regil.log
i=0
for v in default regil default regil; do
  i=$((i+1))
  if [ $v = default ]; then L=$PWD/sfm-project_amd/lib/libsfmcore.so; else L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; fi
  SFMCORE_LIB=$L timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/p$i -o run --output-format csv -- python3 bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/b$i.json 2> $OUT/b$i.err || { tail -20 $OUT/b$i.err; exit 1; }
  f=$(find $OUT/p$i -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$v" "$OUT/b$i.json" <<'PY'
import csv, json, sys
t = {r["Name"].split("(")[0].replace("(anonymous namespace)::", ""): (float(r["TotalDurationNs"]) / 1e6, int(r["Calls"])) for r in csv.DictReader(open(sys.argv[1]))}
k = [v for n, v in t.items() if "reg_hyp_kernel" in n][0]
d = json.loads(open(sys.argv[3]).read().splitlines()[-1]); c = d.get("cfg5", d)
print(sys.argv[2], "reg_hyp ms", round(k[0], 2), "calls", k[1], "register_s", c["stage_s"]["register"], "s/recon", round(c["s_per_reconstruction"], 4), "points", c["points"], "median", c["median_reproj_px"])
PY
done
