set -o pipefail
# Round 5: host-side profile (cProfile) of cfg5 with the BA chunk table off / on: where setup_s goes.
OUT=gpurun_out/q5o; mkdir -p $OUT
export TMPDIR=/tmp
for c in 0 8; do
  SFM_BA_CHUNKS=$c timeout -k 10 400 python -u -m cProfile -o $OUT/c$c.prof bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/c$c.log 2>&1 || { tail -20 $OUT/c$c.log; exit 1; }
  python3 - $OUT/c$c.prof <<'PY'
import pstats, sys
p = pstats.Stats(sys.argv[1])
p.sort_stats("cumulative")
import io
s = io.StringIO(); p.stream = s
p.print_stats("reconstruction.py|sfmcore.py", 25)
print("\n".join(l for l in s.getvalue().splitlines() if l.strip())[:6000])
PY
done
