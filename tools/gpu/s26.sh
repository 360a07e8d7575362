# Round 6: skipping the speculative linearisation where the step is likely the last (the previous
# relative decrease <= ftol^e): e = 0 (always), 0.5, 0.75 — cfg5 interleaved.
set -o pipefail
O=gpurun_out/s26; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in 0 0.5 0.75; do
    SFM_BA_SPEC_SKIP=$v timeout -k 10 600 python bench.py --config cfg5 --steps 2 --warmup 1 > $O/cfg5_skip$v.$r.json 2> $O/cfg5_skip$v.$r.err || { tail -20 $O/cfg5_skip$v.$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/cfg5_skip$v.$r.json').read().splitlines()[-1]); c=d['cfg5']; print('skip=$v', round(c['s_per_reconstruction'],4), c['ba_phase_s']['lm_s'], c['points'], c['median_reproj_px'], c['lm_steps'], c['lm_rejected'], c['cg_iters'])"
  done
done
