set -o pipefail
TAG=$1
bash tools/gpu/run_all.sh $TAG || exit 1
timeout -k 10 900 bash tools/pmc_traffic.sh traffic_$TAG > gpurun_out/traffic_$TAG.log 2>&1 || { tail -5 gpurun_out/traffic_$TAG.log; exit 1; }
grep -A4 "mfma_mutual_kernel\|mutual_finalize" gpurun_out/traffic_$TAG/traffic.json
