# Round 6: the speculative linearisation's policy — every step (1), only after an accepted step
# (acc), never (0) — cfg5 interleaved, with the LM's rejected-step count.
set -o pipefail
O=gpurun_out/s25; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in 1 acc 0; do
    SFM_BA_SPEC=$v timeout -k 10 600 python bench.py --config cfg5 --steps 2 --warmup 1 > $O/cfg5_spec$v.$r.json 2> $O/cfg5_spec$v.$r.err || { tail -20 $O/cfg5_spec$v.$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/cfg5_spec$v.$r.json').read().splitlines()[-1]); c=d['cfg5']; print('spec=$v', round(c['s_per_reconstruction'],4), c['ba_phase_s']['lm_s'], c['points'], c['median_reproj_px'], c['lm_steps'], c['lm_rejected'], c['cg_iters'])"
  done
done
