set -o pipefail
# Round 5: P3P scoring in correspondence slices (REG_SPLIT 4, the default build) against 1 and 8
# slices: registration / incremental tests on the default, then reg_hyp (+ reg_key) time in the
# cfg5 leg, interleaved A/B (rocprofv3 kernel stats).
OUT=gpurun_out/q6s; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_register.py tests/test_gpu_incremental.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
i=0
for v in default split1 split8 default split1 split8; do
  i=$((i+1))
  if [ $v = default ]; then L=$PWD/sfm-project_amd/lib/libsfmcore.so; else L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; fi
  SFMCORE_LIB=$L timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/p$i -o run --output-format csv -- python3 bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/b$i.json 2> $OUT/b$i.err || { tail -20 $OUT/b$i.err; exit 1; }
  python3 - "$OUT/p$i/run_kernel_stats.csv" "$v" "$OUT/b$i.json" <<'PY'
import csv, json, sys
t = {r["Name"]: (float(r["TotalDurationNs"]) / 1e6, int(r["Calls"])) for r in csv.DictReader(open(sys.argv[1]))}
k = sum(v[0] for n, v in t.items() if "reg_hyp_kernel" in n or "reg_key_kernel" in n)
d = json.loads(open(sys.argv[3]).read().splitlines()[-1]); c = d.get("cfg5", d)
print(sys.argv[2], "reg_hyp+key ms", round(k, 2), "register_s", c["stage_s"]["register"], "points", c["points"], "median", c["median_reproj_px"], "registered", c["registered"])
PY
done
