set -o pipefail
# Round 4: PMC of the shipped K1 kernel (mfma_mutual_kernel) at the cfg3 shape (50 x 2048) and at
# K = 4096 (40 images), four counter passes each (tools/pmc_k1.sh).
export TMPDIR=/tmp
timeout -k 10 900 bash tools/pmc_k1.sh r7a_k2048 mfma_mutual > gpurun_out/r7a_k2048.log 2>&1 || { tail -10 gpurun_out/r7a_k2048.log; exit 1; }
tail -30 gpurun_out/r7a_k2048.log
N_IMG=40 K=4096 timeout -k 10 900 bash tools/pmc_k1.sh r7a_k4096 mfma_mutual > gpurun_out/r7a_k4096.log 2>&1 || { tail -10 gpurun_out/r7a_k4096.log; exit 1; }
tail -30 gpurun_out/r7a_k4096.log
