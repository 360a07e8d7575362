set -o pipefail
TAG=$1
bash tools/gpu/k1ab.sh $TAG base pf || exit 1
timeout -k 10 900 bash tools/pmc_k1.sh pmc_$TAG l2fr_scan > /dev/null 2>&1; tail -40 gpurun_out/pmc_$TAG/summary.txt
