set -o pipefail
# Round 5: camera set-up chunk partials in parallel blocks (BA_CAM_SPLIT 1, default build) against
# the chunk loop (variant camsplit0): BA / incremental tests, then the cfg5 leg A/B (rocprofv3).
OUT=gpurun_out/q6t; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ba_lm.py tests/test_gpu_ba_sharded.py tests/test_gpu_incremental.py tests/test_gpu_ba.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
i=0
for v in default camsplit0 default camsplit0; do
  i=$((i+1))
  if [ $v = default ]; then L=$PWD/sfm-project_amd/lib/libsfmcore.so; else L=$PWD/sfm-project_amd/lib/libsfmcore_$v.so; fi
  SFMCORE_LIB=$L timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/p$i -o run --output-format csv -- python3 bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/b$i.json 2> $OUT/b$i.err || { tail -20 $OUT/b$i.err; exit 1; }
  python3 - "$OUT/p$i/run_kernel_stats.csv" "$v" "$OUT/b$i.json" <<'PY'
import csv, json, sys
t = {r["Name"]: (float(r["TotalDurationNs"]) / 1e6, int(r["Calls"])) for r in csv.DictReader(open(sys.argv[1]))}
k = sum(v[0] for n, v in t.items() if "bas_camera_setup" in n or "bas_camera_chunk_part" in n)
d = json.loads(open(sys.argv[3]).read().splitlines()[-1]); c = d.get("cfg5", d)
print(sys.argv[2], "camera set-up ms (whole run)", round(k, 2), "ba_s", c["stage_s"]["bundle_adjust"], "points", c["points"], "median", c["median_reproj_px"], "registered", c["registered"])
PY
done
