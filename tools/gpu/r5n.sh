#!/bin/bash
# PMC record of the K2 fit kernel (cfg3, ordered schedule): VALU activity and waits.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp MODES=0
bash tools/pmc_kernel.sh r5n_pmc_fit "ransac_fit_kernel|ransac_score_kernel" tests/perf/ransac_variants.py
