# Round 6: CG look-ahead depth (SFM_BA_POLL_AHEAD 1 / 2 / 3 / 4 iterations enqueued past a poll
# before the host waits on it) — cfg5 interleaved.
set -o pipefail
O=gpurun_out/s29; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in 2 1 3 4; do
    SFM_BA_POLL_AHEAD=$v timeout -k 10 600 python bench.py --config cfg5 --steps 2 --warmup 1 > $O/cfg5_ahead$v.$r.json 2> $O/cfg5_ahead$v.$r.err || { tail -20 $O/cfg5_ahead$v.$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/cfg5_ahead$v.$r.json').read().splitlines()[-1]); c=d['cfg5']; print('ahead=$v', round(c['s_per_reconstruction'],4), c['ba_phase_s']['lm_s'], c['points'], c['median_reproj_px'], c['lm_steps'], c['cg_iters'])"
  done
done
