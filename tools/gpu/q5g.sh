set -o pipefail
# Round 5: PMC of the group kernel (SFM_K1_GRP=1) and round 4.s kernel (default) at cfg3 and K = 4096.
export TMPDIR=/tmp
export K1_ONLY_BENCH_RULE=1
SFM_K1_GRP=1 timeout -k 10 600 bash tools/pmc_k1.sh q5g_grp_k2048 mfma_mutual_grp > gpurun_out/q5g_grp_k2048.log 2>&1 || { tail -10 gpurun_out/q5g_grp_k2048.log; exit 1; }
SFM_K1_GRP=0 timeout -k 10 600 bash tools/pmc_k1.sh q5g_old_k2048 mfma_mutual_kernel > gpurun_out/q5g_old_k2048.log 2>&1 || { tail -10 gpurun_out/q5g_old_k2048.log; exit 1; }
N_IMG=40 K=4096 SFM_K1_GRP=1 timeout -k 10 600 bash tools/pmc_k1.sh q5g_grp_k4096 mfma_mutual_grp > gpurun_out/q5g_grp_k4096.log 2>&1 || { tail -10 gpurun_out/q5g_grp_k4096.log; exit 1; }
N_IMG=40 K=4096 SFM_K1_GRP=0 timeout -k 10 600 bash tools/pmc_k1.sh q5g_old_k4096 mfma_mutual_kernel > gpurun_out/q5g_old_k4096.log 2>&1 || { tail -10 gpurun_out/q5g_old_k4096.log; exit 1; }
for f in grp_k2048 old_k2048 grp_k4096 old_k4096; do echo "== $f"; tail -25 gpurun_out/q5g_$f.log; done
