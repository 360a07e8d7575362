set -o pipefail
# Round 5: refresh the PMC HBM traffic of the bench kernels (cfg4 and cfg3), one counter per pass.
bash tools/pmc_traffic.sh q6p_cfg4 cfg4 && bash tools/pmc_traffic.sh q6p_cfg3 cfg3
